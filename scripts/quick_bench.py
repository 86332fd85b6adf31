"""Quick single-GPU throughput probe: HIP kernel path vs the PyTorch/MIOpen path.

python scripts/quick_bench.py --arch resnet50 --batch 256 --steps 20
Prints img/s for fwd+bwd(+SGD) of each backend on synthetic data.
"""

import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn.functional as F


def bench_torch(arch, B, steps, warmup, size):
    from imagent_amd.models import resnet
    m = resnet.build(arch).cuda().to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    x = torch.randn(B, 3, size, size, device="cuda").to(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (B,), device="cuda")

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = F.cross_entropy(m(x), y)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / steps
    return B / dt, dt


def bench_hip(arch, B, steps, warmup, size):
    from imagent_amd.models import resnet
    from imagent_amd.models.native import bind_native
    from imagent_amd.ops.misc import XentFn, normalize_u8, sgd_flat
    m = resnet.build(arch)
    st = bind_native(m, "cuda")
    ar = st.arena
    buf = torch.zeros_like(ar.P)
    img = torch.randint(0, 256, (B, size, size, 3), dtype=torch.uint8, device="cuda")
    y = torch.randint(0, 1000, (B,), device="cuda")
    met = torch.zeros(4, device="cuda")
    first = [True]

    def step():
        x = normalize_u8(img, (size, size), 4, (0.5,) * 3, (0.5,) * 3)
        ar.zero_grad()
        loss = XentFn.apply(m(x), y, met, 0.0)
        loss.backward()
        sgd_flat(ar.P, ar.G, buf, ar.S, 0.1, 0.9, 0.0, 1e-4, False, first[0])
        first[0] = False
        st.refresh_shadows()

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / steps
    return B / dt, dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="resnet50")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--size", type=int, default=224)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--which", default="hip,torch")
    a = ap.parse_args()
    for w in a.which.split(","):
        f = bench_hip if w == "hip" else bench_torch
        ips, dt = f(a.arch, a.batch, a.steps, a.warmup, a.size)
        print(f"{w:6s} {a.arch} B={a.batch} {a.size}px: {ips:9.1f} img/s  {dt*1e3:8.2f} ms/step", flush=True)


if __name__ == "__main__":
    main()
