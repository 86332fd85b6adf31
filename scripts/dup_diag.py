"""Per-parameter gradient difference between a B-image step and a 2B-image step whose second half repeats the
first (tests/test_model_gpu.py::test_large_batch_duplicated_halves_match): which layer's backward breaks at the
large batch.   python scripts/dup_diag.py [--batch 1024] [--size 224]"""
import argparse
import copy
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--size", type=int, default=224)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    from imagent_amd.models import resnet
    from imagent_amd.models.native import bind_native
    dev = "cuda"
    torch.manual_seed(21)
    base = resnet.build("resnet50", num_classes=1000)
    g = torch.Generator(device=dev).manual_seed(22)
    x = torch.randn(a.batch, a.size, a.size, 4, device=dev, generator=g).to(torch.bfloat16)
    x[..., 3] = 0
    lab = torch.randint(0, 1000, (a.batch,), device=dev, generator=g)
    out = []
    for dup in (False, True, False):
        model = copy.deepcopy(base)
        st = bind_native(model, dev)
        model.train()
        st.arena.zero_grad()
        xi = torch.cat([x, x]) if dup else x
        li = torch.cat([lab, lab]) if dup else lab
        loss = F.cross_entropy(model(xi), li)
        loss.backward()
        torch.cuda.synchronize()
        out.append((loss.item(), {n: p.grad.float().clone() for n, p in model.named_parameters()}))
        del model, st, xi, li, loss
        torch.cuda.empty_cache()
    (l0, g0), (l1, g1), (l2, g2) = out
    print(f"loss {l0:.6f} vs {l1:.6f} (repeat of the base step: {l2:.6f})")
    print("model order: rel(dup vs base)  rel(base repeat vs base)")
    for n in g0:
        r1 = ((g1[n] - g0[n]).norm() / g0[n].norm().clamp_min(1e-20)).item()
        r2 = ((g2[n] - g0[n]).norm() / g0[n].norm().clamp_min(1e-20)).item()
        if "conv" in n or "fc" in n or "downsample.0" in n:
            print(f"  {n:40s} {r1:9.4f} {r2:9.4f}")
    rows = []
    for n in g0:
        d = ((g1[n] - g0[n]).norm() / g0[n].norm().clamp_min(1e-20)).item()
        rows.append((d, n, g0[n].norm().item(), g1[n].norm().item()))
    for d, n, a0, a1 in sorted(rows, reverse=True)[:a.top]:
        print(f"{d:10.4f}  {n:45s} |g| {a0:.4e} vs {a1:.4e}")
    order = [n for n in g0]
    print("first 10 in model order with rel > 0.05:", [n for n in order if ((g1[n] - g0[n]).norm() / g0[n].norm().clamp_min(1e-20)).item() > 0.05][:10])


if __name__ == "__main__":
    main()
