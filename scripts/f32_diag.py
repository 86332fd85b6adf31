"""Layer-by-layer accuracy of the fp32 kernel path against float64 (and PyTorch fp32 against
float64): where does a whole-model difference come from?

python scripts/f32_diag.py [--size 112 --batch 8]
"""

import argparse
import copy
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn.functional as F


def rel(a, b):
    a, b = a.detach(), b.detach()
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=112)
    ap.add_argument("--batch", type=int, default=8)
    a = ap.parse_args()
    from imagent_amd.data.loader import InputTransform
    from imagent_amd.models import resnet
    from imagent_amd.models.native_f32 import bind_native_f32
    from imagent_amd.ops import f32 as O
    dev = "cuda"
    torch.manual_seed(3)
    ref = resnet.resnet18(num_classes=100).to(dev)
    r64 = copy.deepcopy(ref).double()
    m = resnet.resnet18(num_classes=100)
    m.load_state_dict(ref.state_dict())
    st = bind_native_f32(m, dev)
    u8 = torch.randint(0, 256, (a.batch, a.size, a.size, 3), dtype=torch.uint8, device=dev)
    xr = InputTransform("torch", (a.size, a.size))(u8)
    xh = InputTransform("hip_f32", (a.size, a.size), cpad=4)(u8)
    nchw = lambda t: t.permute(0, 3, 1, 2)
    for mm in (ref, r64, m):
        mm.train()
    acts = {}

    def tap(name, ours, t32, t64):
        acts[name] = (rel(nchw(ours) if ours.dim() == 4 else ours, t64), rel(t32, t64))
        print(f"{name:28s} ours {acts[name][0]:.2e}  torch32 {acts[name][1]:.2e}", flush=True)

    # forward, stage by stage, with autograd on all three
    x32, x64 = xr, xr.double()
    h = O.ConvF32Fn.apply(xh, m.conv1.weight, m.conv1)
    t32 = ref.conv1.forward_torch(x32)
    t64 = r64.conv1.forward_torch(x64)
    tap("stem conv", h, t32, t64)
    h = O.BNF32Fn.apply(h, None, m.bn1, True, st.ws)
    t32 = F.relu(ref.bn1.forward_torch(t32))
    t64 = F.relu(r64.bn1.forward_torch(t64))
    tap("stem bn+relu", h, t32, t64)
    h = O.MaxPoolF32Fn.apply(h, 3, 2, 1)
    t32, t64 = F.max_pool2d(t32, 3, 2, 1), F.max_pool2d(t64, 3, 2, 1)
    tap("maxpool", h, t32, t64)
    inter = []  # (name, ours, t32, t64) intermediate tensors whose gradients are compared

    def keep(name, o, a, b):
        for t in (o, a, b):
            t.retain_grad()
        inter.append((name, o, a, b))

    def tblock(b, x):  # BasicBlock, explicit ops so the intermediates can be kept
        a1 = b.conv1.forward_torch(x)
        b1 = F.relu(b.bn1.forward_torch(a1))
        a2 = b.conv2.forward_torch(b1)
        idt = x if b.downsample is None else b.downsample[1].forward_torch(b.downsample[0].forward_torch(x))
        return a1, b1, a2, F.relu(b.bn2.forward_torch(a2) + idt)

    for bi, (b, b32, b64) in enumerate(zip(m.blocks(), ref.blocks(), r64.blocks())):
        y = h
        a1 = O.ConvF32Fn.apply(y, b.conv1.weight, b.conv1)
        b1 = O.BNF32Fn.apply(a1, None, b.bn1, True, st.ws)
        a2 = O.ConvF32Fn.apply(b1, b.conv2.weight, b.conv2)
        idt = y if b.downsample is None else O.BNF32Fn.apply(
            O.ConvF32Fn.apply(y, b.downsample[0].weight, b.downsample[0]), None, b.downsample[1], False, st.ws)
        h = O.BNF32Fn.apply(a2, idt, b.bn2, True, st.ws)
        r32, r64_ = tblock(b32, t32), tblock(b64, t64)
        for nm, o, q32, q64 in zip(("conv1 out", "bn1 out", "conv2 out", "block out"), (a1, b1, a2, h), r32, r64_):
            keep(f"block {bi} {nm}", o, q32, q64)
        t32, t64 = r32[3], r64_[3]
        tap(f"block {bi}", h, t32, t64)
    p = O.AvgPoolF32Fn.apply(h)
    t32 = torch.flatten(F.adaptive_avg_pool2d(t32, 1), 1)
    t64 = torch.flatten(F.adaptive_avg_pool2d(t64, 1), 1)
    tap("avgpool", p, t32, t64)
    z = O.LinearF32Fn.apply(p, m.fc.weight, m.fc.bias, m.fc)
    t32, t64 = ref.fc.forward_torch(t32), r64.fc.forward_torch(t64)
    tap("logits", z, t32, t64)
    y = torch.randint(0, 100, (a.batch,), device=dev)
    met = torch.zeros(4, device=dev)
    loss = O.XentF32Fn.apply(z, y, met, 0.0)
    l32, l64 = F.cross_entropy(t32, y), F.cross_entropy(t64, y)
    print(f"loss ours {loss.item():.8f} torch32 {l32.item():.8f} f64 {l64.item():.8f}")
    for mm in (m, ref, r64):
        for q in mm.parameters():
            q.grad = torch.zeros_like(q) if mm is not m else q.grad.zero_()
    loss.backward()
    l32.backward()
    l64.backward()
    print("activation gradients: normwise rel error, and rel error of the per-channel row sums")
    for name, o, q32, q64 in inter:
        go, g32_, g64_ = nchw(o.grad), q32.grad, q64.grad
        cs = lambda t: t.double().sum((0, 2, 3))
        print(f"d/d {name:22s} ours {rel(go, g64_):.2e} sum {rel(cs(go), cs(g64_)):.2e}  "
              f"torch32 {rel(g32_, g64_):.2e} sum {rel(cs(g32_), cs(g64_)):.2e}")
    print("ReLU-masked channel sums (= the BN bias gradient) at each bn1: our mask vs float64's")
    for name, o, q32, q64 in inter:
        if not name.endswith("bn1 out"):
            continue
        yo, y64 = nchw(o).double(), q64.double()
        go, g64_ = nchw(o.grad).double(), q64.grad
        mo, m64 = yo > 0, y64 > 0
        cs = lambda g, m: (g * m).sum((0, 2, 3))
        print(f"{name:22s} mask flips {int((mo != m64).sum())} of {mo.numel()}  "
              f"sum(ours g, ours mask) {rel(cs(go, mo), cs(g64_, m64)):.2e}  "
              f"sum(f64 g, ours mask) {rel(cs(g64_, mo), cs(g64_, m64)):.2e}  "
              f"sum(ours g, f64 mask) {rel(cs(go, m64), cs(g64_, m64)):.2e}  "
              f"|sum| / sum|.| {float(cs(g64_, m64).norm() / (g64_ * m64).abs().sum((0, 2, 3)).norm()):.2e}")
    g32 = dict(ref.named_parameters())
    g64 = dict(r64.named_parameters())
    for n, q in m.named_parameters():
        print(f"grad {n:30s} ours {rel(q.grad, g64[n].grad):.2e}  torch32 {rel(g32[n].grad, g64[n].grad):.2e}")


if __name__ == "__main__":
    main()
