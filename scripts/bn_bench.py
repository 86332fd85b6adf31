"""BatchNorm streaming-pass microbenchmark: forward apply and backward apply
for every ResNet-50 BN activation shape, with achieved HBM bandwidth.

python scripts/bn_bench.py --batch 512
Each pass is pure streaming (statistics come from the conv epilogues), so the
target is the HBM roofline: bytes moved / ~6 TB/s.
"""

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch


def timeit(fn, reps=20, warm=3):
    for _ in range(warm):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    a = ap.parse_args()
    from imagent_amd.models.resnet import BatchNorm2d, BNWork
    from imagent_amd.ops import _lib
    from imagent_amd.ops.bn import bn_apply_backward, bn_fwd_launch
    dev = "cuda"
    B = a.batch
    # (C, H, mode, count per step): R50 BN sites at 224
    sites = [(64, 112, 0, 1), (64, 56, 0, 6), (256, 56, 1, 2), (256, 56, 2, 1),
             (128, 56, 0, 1), (128, 28, 0, 7), (512, 28, 1, 3), (512, 28, 2, 1),
             (256, 28, 0, 1), (256, 14, 0, 11), (1024, 14, 1, 5), (1024, 14, 2, 1),
             (512, 14, 0, 1), (512, 7, 0, 5), (2048, 7, 1, 2), (2048, 7, 2, 1)]
    S = _lib.STAT_SLOTS
    nbw = _lib.kernels().imk_bn_bwd_scratch_floats(1)

    def mk(C):
        bn = BatchNorm2d(C).to(dev)
        bn.weight.grad = torch.zeros_like(bn.weight)
        bn.bias.grad = torch.zeros_like(bn.bias)
        slab = torch.zeros(S, 2, C, device=dev)
        slab[0, 0] = 1.0
        slab[0, 1] = 4.0
        bn.work = BNWork(slab, torch.tensor([[0.0] * C, [1.0] * C], device=dev), torch.ones(2, C, device=dev),
                         torch.zeros(nbw * C, device=dev))
        return bn

    # achievable streaming rate on this box: a 2-stream copy and a 3-stream add of the layer-1 activation size
    ra = torch.randn(B, 56, 56, 64, device=dev).to(torch.bfloat16)
    rb, rc = torch.randn_like(ra), torch.empty_like(ra)
    nb0 = ra.numel() * 2
    tc = timeit(lambda: rc.copy_(ra))
    tadd = timeit(lambda: torch.add(ra, rb, out=rc))
    print(f"reference: copy {nb0 * 2 / tc / 1e6:.2f} TB/s, add (2 in, 1 out) {nb0 * 3 / tadd / 1e6:.2f} TB/s "
          f"({nb0 / 1e6:.0f} MB per tensor)")
    del ra, rb, rc
    tot_f = tot_b = tot_rf = tot_rb = 0.0
    print(f"{'C':>5} {'H':>4} mode cnt | {'fwd us':>8} {'TB/s':>5} | {'bwd us':>8} {'TB/s':>5}")
    for C, H, mode, cnt in sites:
        x = torch.randn(B, H, H, C, device=dev).to(torch.bfloat16)
        x2 = torch.randn_like(x) if mode else None
        y = torch.empty_like(x)
        bn, bn2 = mk(C), (mk(C) if mode == 2 else None)
        nb = x.numel() * 2
        tf = timeit(lambda: bn_fwd_launch(x, bn.work.stats, bn.weight, bn.bias, y, bn.work.save, x2=x2,
                                          stats2=bn2.work.stats if bn2 else None,
                                          gamma2=bn2.weight if bn2 else None, beta2=bn2.bias if bn2 else None,
                                          save2=bn2.work.save if bn2 else None, mode=mode, relu=True))
        bf = nb * (3 if mode else 2)  # x (+x2|res) read, y written
        g = torch.randn_like(x)
        tb = timeit(lambda: bn_apply_backward(g, x, x2 if mode == 2 else None, bn, bn2, mode))
        bb = nb * (3 + (2 if mode == 2 else 0))  # g, x read, dx written (+x2 read, dx2 written)
        print(f"{C:5d} {H:4d} {mode:4d} {cnt:3d} | {tf:8.1f} {bf / tf / 1e6:5.2f} | {tb:8.1f} {bb / tb / 1e6:5.2f}",
              flush=True)
        tot_f += tf * cnt
        tot_b += tb * cnt
        tot_rf += bf / 6e6 * cnt
        tot_rb += bb / 6e6 * cnt
        del x, x2, y, g
    print(f"per step: fwd {tot_f:.0f} us (roof {tot_rf:.0f}), bwd apply {tot_b:.0f} us (roof {tot_rb:.0f})")


if __name__ == "__main__":
    main()
