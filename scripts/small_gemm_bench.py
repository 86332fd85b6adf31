"""Timing of the small fp32 GEMMs around the Gram-form bn3 (ops/bn_gram.py): Q = (W3^T diag(B)) W3 [p][p]
over K = 4p, P = W3 G [4p][p] over K = p, per ResNet-50 stage, for the operand layouts torch.mm can be
handed (hipBLASLt picks its kernel by layout and shape).

python scripts/small_gemm_bench.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch


def timeit(fn, reps=50, warm=5):
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
    dev = torch.device("cuda")
    for p in (64, 128, 256, 512):
        C4 = 4 * p
        wt = torch.randn(p, C4, device=dev)  # W3^T as the dgrad sees it ([p][4p])
        b = torch.randn(C4, device=dev)
        ref = (wt.double() * b.double()) @ wt.double().t()
        cands = {
            "mm(A, W^T view)": lambda: torch.mm(wt * b, wt.t()),
            "mm(A, W^T contig)": lambda: torch.mm(wt * b, wt.t().contiguous()),
            "matmul bmm-1": lambda: torch.matmul((wt * b).unsqueeze(0), wt.t().unsqueeze(0))[0],
            "mm(W view^T.., ) as (W^T B W)": lambda: torch.mm(wt.t().contiguous().t() * b, wt.t()),
            "einsum": lambda: torch.einsum("ik,jk->ij", wt * b, wt),
        }
        line = f"Q p={p:3d}:"
        for k, f in cands.items():
            err = ((f().double() - ref).norm() / ref.norm()).item()
            line += f" | {k} {timeit(f):7.1f} us e{err:.0e}"
        print(line, flush=True)


if __name__ == "__main__":
    main()
