"""Isolated timing of the stem pool's fused passes (ops/misc.py StemFn): the BN + ReLU + 3x3/2 max-pool forward
(imk_maxpool_fwd_bn, with the argmax-input copy xsel) and the quad-gather backward that stores the ReLU-masked BN
upstream gradient and reduces the BN sums (imk_maxpool_bwd_bnr), ResNet-50 stem shapes at --batch images.
us per call and HBM TB/s over the bytes each pass must move (inputs once, outputs once).
IMAGENT_POOL_NT=0 / 1 selects the backward's plain / non-temporal (default) stores (A/B: one run per setting).

python scripts/pool_bench.py [--batch 4096]
"""

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch


def timeit(fn, reps=10, warm=2):
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
    ap.add_argument("--batch", type=int, default=4096)
    args = ap.parse_args()
    from imagent_amd.ops import _lib
    k = _lib.kernels()
    dev = torch.device("cuda")
    N, H, C = args.batch, 112, 64
    OH = 56
    torch.manual_seed(0)
    x = torch.randn(N, H, H, C, device=dev).to(torch.bfloat16)
    sums = torch.zeros(2, C, device=dev)
    sums[1] = 1.0  # (mean 0, variance 1)
    gamma = torch.ones(C, device=dev)
    beta = torch.zeros(C, device=dev)
    save = torch.zeros(2, C, device=dev)
    y = torch.empty(N, OH, OH, C, device=dev, dtype=torch.bfloat16)
    idx = torch.empty(N, OH, OH, C, device=dev, dtype=torch.uint8)
    xsel = torch.empty_like(y)
    st = _lib.stream_ptr()

    def fwd():
        _lib.check(k.imk_maxpool_fwd_bn(x.data_ptr(), sums.data_ptr(), gamma.data_ptr(), beta.data_ptr(),
                                        save.data_ptr(), y.data_ptr(), idx.data_ptr(), xsel.data_ptr(), N, H, H, C,
                                        OH, OH, 3, 2, 1, 1e-5, st), "pool fwd")
    fwd()
    dy = torch.randn_like(y)
    g = torch.empty_like(x)
    slab = torch.zeros(k.imk_bn_bwd_scratch_floats(C), device=dev)  # the BN's backward scratch

    def bwd():
        _lib.check(k.imk_maxpool_bwd_bnr(dy.data_ptr(), idx.data_ptr(), g.data_ptr(), x.data_ptr(), xsel.data_ptr(),
                                         save.data_ptr(), gamma.data_ptr(), beta.data_ptr(), slab.data_ptr(), N, H, H,
                                         C, OH, OH, 3, 2, 1, st), "pool bwd")
    xb, yb = x.numel() * 2, y.numel() * 2
    tf = timeit(fwd)
    tb = timeit(bwd)
    fb = xb + 2 * yb + yb // 2        # x in; y, xsel, idx out
    bb = 2 * yb + yb // 2 + xb        # dy, xsel, idx in; g out
    print(f"batch {N} pool_nt={os.environ.get('IMAGENT_POOL_NT', '1')}: fwd {tf:8.1f} us {fb / tf / 1e6:5.2f} TB/s | "
          f"bwd {tb:8.1f} us {bb / tb / 1e6:5.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
