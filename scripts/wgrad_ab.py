"""Weight-gradient kernel A/B on the R50 shapes the default dispatch leaves on the register-staged loop (3x3 stride 2,
3x3 at 7x7) and on the Ci = 64 1x1 shapes: isolated time per call for variant -1 (register-staged wgrad_kernel),
1..4 (LDS-DMA wgrad_v3 stage shapes), 6 (its 256 x 256 tile), 9 (halo-tiled) and 0 (default dispatch), batch 1024, bf16.

    python scripts/wgrad_ab.py [--batch 1024] [--variants 0,-1,1,2,4]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (Ci, H, Co, k, s, calls per step at R50)
SHAPES = [(128, 56, 128, 3, 2, 1), (256, 28, 256, 3, 2, 1), (512, 14, 512, 3, 2, 1), (512, 7, 512, 3, 1, 2),
          (64, 56, 256, 1, 1, 4), (64, 56, 64, 1, 1, 1), (256, 56, 64, 1, 1, 2), (64, 56, 64, 3, 1, 3), (128, 28, 128, 3, 1, 3)]
# every R50 1x1 wgrad with Ci, Co >= 128 (--set 1x1): the wide-tile variant 6
SHAPES_1X1 = [(256, 56, 128, 1, 1, 1), (128, 28, 512, 1, 1, 4), (512, 28, 128, 1, 1, 3), (256, 56, 512, 1, 2, 1),
              (512, 28, 256, 1, 1, 1), (256, 14, 1024, 1, 1, 6), (1024, 14, 256, 1, 1, 5), (512, 28, 1024, 1, 2, 1),
              (1024, 14, 512, 1, 1, 1), (512, 7, 2048, 1, 1, 3), (2048, 7, 512, 1, 1, 2), (1024, 14, 2048, 1, 2, 1)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--variants", default="0,-1,1,2,4,9")
    ap.add_argument("--set", default="default", choices=["default", "1x1"])
    ap.add_argument("--only", default=None, help="Ci,H,Co,k,s of one shape")
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    from imagent_amd.ops.conv import igemm_wgrad
    dev = "cuda"
    # clock ramp: the first ~second of GPU work runs 10-15 % slower (round-5 A/Bs timed the first config slowest),
    # so spin the GPU before the first timed call
    _a = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
    for _ in range(200):
        _a = _a @ _a.T * 1e-4
    torch.cuda.synchronize()
    variants = [int(v) for v in a.variants.split(",")]
    print("   Ci    H   Co k s | n | " + " | ".join(f"v{v:>3} us" for v in variants))
    tot = [0.0] * len(variants)
    for ci, h, co, k, s, n in (SHAPES_1X1 if a.set == "1x1" else SHAPES):
        if a.only and tuple(int(v) for v in a.only.split(",")) != (ci, h, co, k, s):
            continue
        oh = (h + 2 * (k // 2) - k) // s + 1
        x = torch.randn(a.batch, h, h, ci, device=dev).to(torch.bfloat16)
        dy = torch.randn(a.batch, oh, oh, co, device=dev).to(torch.bfloat16)
        dw = torch.zeros(co, k * k * ci, device=dev)
        row = []
        ref = None
        for v in variants:
            try:
                for _ in range(2):
                    dw.zero_()
                    igemm_wgrad(dy, x, dw, s, k // 2, k, k, variant=v)
                torch.cuda.synchronize()
                if ref is None:
                    ref = dw.clone()
                err = ((dw - ref).norm() / ref.norm()).item()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                reps = a.reps
                e0.record()
                for _ in range(reps):
                    igemm_wgrad(dy, x, dw, s, k // 2, k, k, variant=v)
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) / reps * 1e3
                row.append(f"{us:7.1f}{'' if err < 1e-2 else '!'}")
                tot[variants.index(v)] += us * n
            except Exception as ex:  # a variant that does not cover the shape
                row.append("    n/a" if "-106" in str(ex) else "    err")
        print(f"{ci:5d} {h:4d} {co:4d} {k} {s} | {n} | " + " | ".join(f"{r:>8}" for r in row), flush=True)
    print("per step (us, x calls; n/a counted as 0): " + " | ".join(f"v{v} {t:.0f}" for v, t in zip(variants, tot)))


if __name__ == "__main__":
    main()
