"""Isolated timing of layer 1's conv3 dgrad family (K = 256 -> 64 channels at 56x56) on the streaming 1x1
kernel: plain, with bn2's BN-backward epilogue (mask + sums from x), and the Gram form over [g | h2]
(ops/bn_gram.py gram_dgrad) -- to separate the kernel's own speed from in-step contention.

python scripts/gram_dgrad_bench.py --batch 2048
"""

import argparse
import os
import sys
import types

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    from imagent_amd.models.resnet import BatchNorm2d, BNWork
    from imagent_amd.ops import _lib
    from imagent_amd.ops.bn_gram import GramBN, gram_dgrad
    from imagent_amd.ops.conv import BNBwdFuse, igemm_dgrad
    dev = torch.device("cuda:0")
    N, H, C4, p = a.batch, 56, 256, 64
    torch.manual_seed(0)
    g = torch.randn(N, H, H, C4, device=dev).to(torch.bfloat16)
    h2 = torch.randn(N, H, H, p, device=dev).to(torch.bfloat16)
    x = torch.randn(N, H, H, p, device=dev).to(torch.bfloat16)
    wt = (torch.randn(p, 1, 1, C4, device=dev) / 16).to(torch.bfloat16)
    nbw = _lib.kernels().imk_bn_bwd_scratch_floats(1)
    bn = BatchNorm2d(p).to(dev)
    save = torch.stack([torch.randn(p, device=dev) * 0.1, torch.rand(p, device=dev) + 0.5])
    bn.work = BNWork(None, None, save, torch.zeros(nbw * p, device=dev))
    conv = types.SimpleNamespace(wt_bf16=wt, kh=1, stride=1)
    gb = GramBN(g, torch.randn(3, C4, device=dev) * 0.01)
    spin = torch.randn(4096, 4096, device=dev)
    for _ in range(30):  # clocks up
        spin = spin @ spin
        spin /= spin.norm()
    torch.cuda.synchronize()
    M = N * H * H
    cases = {
        "plain": lambda: igemm_dgrad(g, wt, (H, H), 1, 0, 1, 1),
        "bnb_x": lambda: igemm_dgrad(g, wt, (H, H), 1, 0, 1, 1, bnb=BNBwdFuse(x, bn)),
        "gram_bnb_x": lambda: gram_dgrad(gb, conv, h2, BNBwdFuse(x, bn)),
    }
    nbytes = {"plain": M * (C4 + p) * 2, "bnb_x": M * (C4 + 2 * p) * 2, "gram_bnb_x": M * (C4 + 3 * p) * 2}
    for name, fn in cases.items():
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
        print(f"{name:12s} {us:8.1f} us  {nbytes[name] / us / 1e6:5.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
