"""Does a training step at 4096 img/GPU (layer-1 activations and the stem output past 2^31 elements) compute the
same gradients as at 2048? A duplicated batch cat([b, b]) has b's batch statistics and, under a mean loss, b's
weight gradients. Reports per-parameter relative differences for: 2048 vs 2048 again (the float-atomic noise floor)
and 4096 (duplicated) vs 2048, on a shallow bottleneck net (blocks [3, 1, 1, 1]: less chaotic amplification than
ResNet-50's 16 blocks) and optionally ResNet-50.

    python scripts/dup4096_check.py [--arch shallow|resnet50] [--batch 2048]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="shallow")
    ap.add_argument("--batch", type=int, default=2048)
    a = ap.parse_args()
    from imagent_amd.models import resnet
    from imagent_amd.models.native import bind_native
    from imagent_amd.ops.misc import XentFn, normalize_u8
    dev = torch.device("cuda")
    torch.manual_seed(0)
    m = resnet.ResNet(resnet.Bottleneck, [3, 1, 1, 1]) if a.arch == "shallow" else resnet.resnet50()
    st = bind_native(m, dev)
    m.train()
    B = a.batch
    img = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, device=dev)
    lab = torch.randint(0, 1000, (B,), device=dev)
    mean, std = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)
    names = [n for n, _ in m.named_parameters()]
    pick = [n for n in names if n.endswith("weight")]
    pick = pick[:4] + pick[len(pick) // 2:len(pick) // 2 + 2] + pick[-3:]

    def step(images, labels):
        st.arena.G.zero_()
        met = torch.zeros(4, device=dev)
        loss = XentFn.apply(m(normalize_u8(images, (224, 224), 4, mean, std)), labels, met, 0.0)
        loss.backward()
        torch.cuda.synchronize()
        g = {n: p.grad.detach().float().clone() for n, p in m.named_parameters() if n in pick}
        lv = loss.item()
        del loss
        torch.cuda.empty_cache()
        return lv, g

    l1, g1 = step(img, lab)
    l1b, g1b = step(img, lab)
    l2, g2 = step(torch.cat([img, img]), torch.cat([lab, lab]))
    print(f"loss {B}: {l1:.6f} / again {l1b:.6f} / {2 * B} duplicated {l2:.6f}")
    rel = lambda u, v: ((u - v).norm() / v.norm().clamp_min(1e-30)).item()  # noqa: E731
    worst = 0.0
    for n in pick:
        floor, d = rel(g1b[n], g1[n]), rel(g2[n], g1[n])
        worst = max(worst, d / max(floor, 1e-6))
        print(f"{n:40s} noise floor {floor:.2e}  {2 * B} dup vs {B} {d:.2e}")
    print(f"worst ratio (dup diff / noise floor) {worst:.1f}")


if __name__ == "__main__":
    main()
