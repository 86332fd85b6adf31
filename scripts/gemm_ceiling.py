"""Library-GEMM ceiling for the R50 conv shapes: hipBLASLt (torch.mm, bf16) on the dense GEMM each
conv lowers to (M = N*OH*OW pixels, N = Cout, K = taps*Cin) -- what a plain, pre-gathered GEMM of
the same size reaches on this chip, to set the conv kernels' targets against.

python scripts/gemm_ceiling.py [--batch 1024]
"""

import argparse

import torch


def timeit(fn, reps=10, warm=3):
    for _ in range(warm):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    a = ap.parse_args()
    B = a.batch
    # (Cin, H_out, Cout, k): fwd GEMM M = B*H*H, N = Cout, K = k*k*Cin
    shapes = [(64, 56, 64, 3), (128, 28, 128, 3), (256, 14, 256, 3), (512, 7, 512, 3),
              (64, 56, 256, 1), (256, 56, 64, 1), (512, 28, 128, 1), (128, 28, 512, 1),
              (1024, 14, 256, 1), (256, 14, 1024, 1), (2048, 7, 512, 1), (512, 7, 2048, 1)]
    print(f"{'Cin':>5} {'H':>4} {'Cout':>5} k | {'M':>8} {'N':>5} {'K':>5} | {'us':>8} {'TF/s':>6} | NT-layout us")
    for ci, h, co, k in shapes:
        M, N, K = B * h * h, co, k * k * ci
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
        t = timeit(lambda: torch.mm(x, w.t()))
        wt = w.t().contiguous()
        t2 = timeit(lambda: torch.mm(x, wt))
        print(f"{ci:5d} {h:4d} {co:5d} {k} | {M:8d} {N:5d} {K:5d} | {t:8.1f} {2 * M * N * K / t / 1e6:6.0f} | {t2:8.1f}",
              flush=True)
        del x, w, wt


if __name__ == "__main__":
    main()
