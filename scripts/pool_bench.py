"""Stand-alone timing of the stem pool's fused passes at the training shape (2048 x 112 x 112 x 64 -> 56 x 56):
imk_maxpool_fwd_bn (with the per-window argmax input) and imk_maxpool_bwd_bnr from it.

python scripts/pool_bench.py --batch 2048
"""

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    from imagent_amd.ops import _lib
    k = _lib.kernels()
    dev = torch.device("cuda:0")
    N, H, C, OH = a.batch, 112, 64, 56
    x = torch.randn(N, H, H, C, device=dev).to(torch.bfloat16)
    sums = torch.stack([torch.zeros(C, device=dev), torch.ones(C, device=dev)]).contiguous()
    gamma, beta = torch.ones(C, device=dev), torch.zeros(C, device=dev)
    save = torch.empty(2, C, device=dev)
    y = torch.empty(N, OH, OH, C, device=dev, dtype=torch.bfloat16)
    idx = torch.empty(y.shape, device=dev, dtype=torch.uint8)
    xsel = torch.empty_like(y)
    dy = torch.randn(y.shape, device=dev).to(torch.bfloat16)
    g = torch.empty_like(x)
    slab = torch.zeros(32, 3, C, device=dev)
    st = _lib.stream_ptr()
    spin = torch.randn(4096, 4096, device=dev)
    for _ in range(30):
        spin = spin @ spin
        spin /= spin.norm()

    def fwd():
        _lib.check(k.imk_maxpool_fwd_bn(x.data_ptr(), sums.data_ptr(), gamma.data_ptr(), beta.data_ptr(),
                                        save.data_ptr(), y.data_ptr(), idx.data_ptr(), xsel.data_ptr(), N, H, H, C,
                                        OH, OH, 3, 2, 1, 1e-5, st), "fwd")

    def bwd():
        _lib.check(k.imk_maxpool_bwd_bnr(dy.data_ptr(), idx.data_ptr(), g.data_ptr(), x.data_ptr(), xsel.data_ptr(),
                                         save.data_ptr(), gamma.data_ptr(), beta.data_ptr(), slab.data_ptr(), N, H,
                                         H, C, OH, OH, 3, 2, 1, st), "bwd")
    big = N * H * H * C * 2
    nb = big + big // 4 * 2 + big // 8  # fwd: x in, y + xsel + idx out; bwd: g out, dy + xsel + idx in
    for name, fn in (("pool_fwd_bn", fwd), ("pool_bwd_bnr", bwd)):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1000 / a.reps
        print(f"{name:14s} {us:8.1f} us  {nb / us / 1e6:5.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
