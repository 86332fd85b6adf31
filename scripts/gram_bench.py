"""Isolated timing of the skinny 1x1 weight-gradient GEMMs of the Gram-form bn3 (ops/bn_gram.py):
T = g^T h2 ([4p][p] over M pixels, on the main stream before conv3's dgrad) and G = h2^T h2 ([p][p], in the
forward before conv3's epilogue), ResNet-50 at --batch images. Every wgrad variant of ops.conv.igemm_wgrad
(0 default dispatch, -1 register-staged, 1..4 the v3 LDS-DMA stage shapes, 9 the gram kernel) and
torch.mm (hipBLASLt) as reference; us per call and effective HBM TB/s (operand bytes read once).

python scripts/gram_bench.py [--batch 1024] [--variants 0,-1,1,2,3,4]
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
    return s.elapsed_time(e) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--variants", default="0,-1,1,2,3,4")
    ap.add_argument("--splits", default="0", help="split-K counts to try (0: the kernel's own choice)")
    args = ap.parse_args()
    from imagent_amd.ops.conv import igemm_wgrad
    B = args.batch
    dev = torch.device("cuda")
    shapes = []
    for hw, p in ((56, 64), (28, 128), (14, 256), (7, 512)):
        shapes.append((f"T  {4 * p}x{p} @{hw}", hw, 4 * p, p))
        shapes.append((f"G  {p}x{p} @{hw}", hw, p, p))
    variants = [int(v) for v in args.variants.split(",")]
    splits = [int(v) for v in args.splits.split(",")]
    for label, hw, co, ci in shapes:
        M = B * hw * hw
        torch.manual_seed(0)
        x = torch.randn(B, hw, hw, ci, device=dev).to(torch.bfloat16)
        dy = x if co == ci else torch.randn(B, hw, hw, co, device=dev).to(torch.bfloat16)
        ref = torch.mm(dy.view(M, co).t().float(), x.view(M, ci).float())
        gb = (M * co * 2 + (0 if dy is x else M * ci * 2)) / 1e9
        out = torch.zeros(co, ci, device=dev)
        line = f"{label:22s} M {M:8d} {gb:6.3f} GB |"
        t = timeit(lambda: torch.mm(dy.view(M, co).t(), x.view(M, ci)))
        line += f" mm {t:7.1f} us {gb / t * 1e3:5.2f} TB/s |"
        if co == ci:  # the symmetric Gram path (ops/bn_gram.py gram_G)
            from imagent_amd.ops.bn_gram import gram_G
            out.zero_()
            gram_G(x, out)
            t = timeit(lambda: gram_G(x, out))
            out.zero_()
            gram_G(x, out)
            e = ((out - ref).norm() / ref.norm()).item()
            line += f" gramG {t:7.1f} us {gb / t * 1e3:5.2f} TB/s e{e:.0e} |"
        for v in variants:
            for sp in splits:
                tag = f"v{v}" + (f"/s{sp}" if sp else "")
                try:
                    out.zero_()
                    igemm_wgrad(dy, x, out, 1, 0, 1, 1, splits=sp, variant=v)
                    torch.cuda.synchronize()
                    err = (out - ref).norm().item() / ref.norm().item()
                    t = timeit(lambda: igemm_wgrad(dy, x, out, 1, 0, 1, 1, splits=sp, variant=v))
                    line += f" {tag} {t:6.1f} us {gb / t * 1e3:4.2f} TB/s e{err:.0e} |"
                except Exception:  # shape not covered by this variant
                    line += f" {tag} n/a |"
        print(line, flush=True)


if __name__ == "__main__":
    main()
