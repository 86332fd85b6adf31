"""Per-layer conv microbenchmark: HIP kernels (fwd / dgrad / wgrad) vs MIOpen.

python scripts/conv_bench.py --arch resnet50 --batch 256 [--miopen]
Prints one line per unique conv shape with time, TFLOP/s and the HBM roofline
time (operand + result bytes at 6 TB/s) so the optimisation target is clear.
"""

import argparse
import collections
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn.functional as F


def shapes(arch, B, size):
    from imagent_amd.models import resnet
    m = resnet.build(arch)
    out = collections.OrderedDict()
    h = size // 2  # after stem conv
    # walk the forward to get input spatial sizes
    hw = {}
    x = size

    def add(conv, H):
        key = (conv.in_channels, H, conv.out_channels, conv.kh, conv.stride, conv.padding)
        out[key] = out.get(key, 0) + 1

    add(m.conv1, size)
    H = (size + 1) // 2 // 2 + (0 if size % 4 else 0)
    H = ((size + 6 - 7) // 2 + 1 + 2 - 3) // 2 + 1
    for b in m.blocks():
        Hin = H
        for conv, _, _ in b.convs_bns():
            add(conv, H)
            H = (H + 2 * conv.padding - conv.kh) // conv.stride + 1
        if b.downsample is not None:
            add(b.downsample[0], Hin)
    return out


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
    return s.elapsed_time(e) / reps * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="resnet50")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--size", type=int, default=224)
    ap.add_argument("--miopen", action="store_true")
    ap.add_argument("--blas", action="store_true",
                    help="also time the plain-GEMM equivalent (torch.matmul -> hipBLASLt) of 1x1 stride-1 convs")
    ap.add_argument("--json", default=None)
    ap.add_argument("--only", default=None, help="Ci,H,Co,k,s of one shape")
    ap.add_argument("--no-stats", action="store_true", help="forward without the fused BN statistics")
    ap.add_argument("--epi", type=int, default=0, help="0 auto, 1 direct, 2 LDS-staged epilogue")
    ap.add_argument("--fp8", action="store_true", help="also time the fp8 (e4m3, block-scaled MFMA) forward")
    ap.add_argument("--tiles", default=None, help="comma list of explicit tile ids to time for fwd/dgrad")
    ap.add_argument("--bnb", action="store_true",
                    help="also time the dgrad with the fused BatchNorm-backward epilogue (ReLU mask bits, "
                         "the model's block-output form), for the auto tile and every --tiles id")
    a = ap.parse_args()
    from imagent_amd.ops.conv import conv_out_size, igemm_dgrad, igemm_fwd, igemm_wgrad
    dev = "cuda"
    tot = collections.defaultdict(float)
    # clock ramp: the first ~second of GPU work runs 10-15 % slower (round-5 A/Bs timed the first config slowest),
    # so spin the GPU before the first timed call
    _a = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
    for _ in range(200):
        _a = _a @ _a.T * 1e-4
    torch.cuda.synchronize()
    rows = []
    print(f"{'Ci':>5} {'H':>4} {'Co':>5} k s | cnt | {'fwd us':>8} {'TF':>6} {'roof':>6} | {'dgrad':>8} {'TF':>6} | "
          f"{'wgrad':>8} {'TF':>6}" + (" | miopen fwd" if a.miopen else ""))
    for (Ci, H, Co, k, s, p), cnt in shapes(a.arch, a.batch, a.size).items():
        if a.only and tuple(int(v) for v in a.only.split(",")) != (Ci, H, Co, k, s):
            continue
        stem = Ci == 3
        Cin = 4 if stem else Ci
        B = a.batch
        OH = conv_out_size(H, k, s, p)
        x = torch.randn(B, H, H, Cin, device=dev).to(torch.bfloat16)
        w = (torch.randn(Co, k, k, Cin, device=dev) * 0.05).to(torch.bfloat16)
        if stem:
            w = torch.zeros(Co, k, 32, device=dev, dtype=torch.bfloat16)
        wt = w.permute(3, 1, 2, 0).contiguous() if not stem else None
        dy = torch.randn(B, OH, OH, Co, device=dev).to(torch.bfloat16)
        dw = torch.zeros(Co, k, 32, device=dev) if stem else torch.zeros(Co, k, k, Cin, device=dev)
        stats = None if a.no_stats else torch.zeros(32, 2, Co, device=dev)
        flops = 2.0 * B * OH * OH * Co * k * k * Ci
        t_f = timeit(lambda: igemm_fwd(x, w, s, p, k, k, stats=stats, stem=stem, epi=0 if stem else a.epi))
        t_d = timeit(lambda: igemm_dgrad(dy, wt, (H, H), s, p, k, k, epi=a.epi)) if not stem else 0.0
        t_w = timeit(lambda: igemm_wgrad(dy, x, dw, s, p, k, k, stem=stem))
        roof = (x.numel() * 2 + dy.numel() * 2 + w.numel() * 2) / 6e12 * 1e6
        line = (f"{Ci:5d} {H:4d} {Co:5d} {k} {s} | {cnt:3d} | {t_f:8.1f} {flops / t_f / 1e6:6.0f} {roof:6.1f} | "
                f"{t_d:8.1f} {flops / max(t_d, 1e-9) / 1e6:6.0f} | {t_w:8.1f} {flops / t_w / 1e6:6.0f}")
        r = dict(Ci=Ci, H=H, Co=Co, k=k, s=s, cnt=cnt, fwd_us=t_f, dgrad_us=t_d, wgrad_us=t_w, gflop=flops / 1e9,
                 roof_us=roof)
        if a.miopen:
            xc = x[..., :Ci].permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
            wc = (torch.randn(Co, Ci, k, k, device=dev) * 0.05).to(torch.bfloat16).contiguous(
                memory_format=torch.channels_last)
            t_m = timeit(lambda: F.conv2d(xc, wc, None, s, p))
            line += f" | {t_m:8.1f}"
            r["miopen_fwd_us"] = t_m
        if a.blas and k == 1 and s == 1 and not stem:
            x2, w2, dy2 = x.view(-1, Ci), w.view(Co, Ci), dy.view(-1, Co)
            t_bf = timeit(lambda: torch.matmul(x2, w2.t()))
            t_bd = timeit(lambda: torch.matmul(dy2, w2))
            t_bw = timeit(lambda: torch.matmul(dy2.t(), x2))
            line += (f" | blas fwd {t_bf:7.1f} dgrad {t_bd:7.1f} wgrad {t_bw:7.1f} "
                     f"({flops / t_bf / 1e6:5.0f}/{flops / t_bd / 1e6:5.0f}/{flops / t_bw / 1e6:5.0f} TF)")
            r["blas_us"] = (t_bf, t_bd, t_bw)
            tot["blas_fwd"] += t_bf * cnt
            tot["blas_dgrad"] += t_bd * cnt
            tot["blas_wgrad"] += t_bw * cnt
            tot["hip_1x1_fwd"] += t_f * cnt
            tot["hip_1x1_dgrad"] += t_d * cnt
            tot["hip_1x1_wgrad"] += t_w * cnt
        if a.fp8 and not stem and Ci % 16 == 0:
            x8 = x.float().clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8)
            w8 = w.float().to(torch.float8_e4m3fn).view(torch.uint8)
            e8 = torch.zeros(2, dtype=torch.int32, device=dev)
            t8 = timeit(lambda: igemm_fwd(x8, w8, s, p, k, k, stats=stats, fp8=(e8[0:1], e8[1:2])))
            line += f" | fp8 fwd {t8:8.1f} {flops / t8 / 1e6:6.0f}"
            r["fp8_fwd_us"] = t8
            tot["fp8_fwd"] += t8 * cnt
            if Co % 16 == 0:  # dgrad: e5m2 gradient x e4m3 transposed weights
                g8 = dy.float().to(torch.float8_e5m2).view(torch.uint8)
                wt8 = wt.float().to(torch.float8_e4m3fn).view(torch.uint8)
                f8d = (g8, e8[0:1], wt8, e8[1:2])
                t8d = timeit(lambda: igemm_dgrad(dy, wt8, (H, H), s, p, k, k, fp8=f8d))
                line += f" | fp8 dgrad {t8d:8.1f} {flops / t8d / 1e6:6.0f}"
                r["fp8_dgrad_us"] = t8d
                tot["fp8_dgrad"] += t8d * cnt
        bnb = None
        if a.bnb and not stem and Ci % 8 == 0 and k >= s:
            from imagent_amd.models.resnet import BatchNorm2d, BNWork
            from imagent_amd.ops import _lib
            from imagent_amd.ops.bn import relu_mask_bits
            from imagent_amd.ops.conv import BNBwdFuse
            bn = BatchNorm2d(Ci).to(dev)
            xb = torch.randn(B, H, H, Ci, device=dev).to(torch.bfloat16)
            save = torch.stack([xb.float().reshape(-1, Ci).mean(0), torch.ones(Ci, device=dev)])
            bn.work = BNWork(torch.zeros(_lib.STAT_SLOTS, 2, Ci, device=dev), torch.zeros(2, Ci, device=dev), save,
                             torch.zeros(_lib.kernels().imk_bn_bwd_scratch_floats(Ci), device=dev))
            bits = relu_mask_bits(torch.relu(torch.randn_like(xb)))
            bnb = BNBwdFuse(xb, bn, y=bits)
            t_b = timeit(lambda: igemm_dgrad(dy, wt, (H, H), s, p, k, k, bnb=bnb))
            line += f" | dgrad+bnb {t_b:8.1f} ({flops / t_b / 1e6:5.0f} TF)"
            r["dgrad_bnb_us"] = t_b
            tot["dgrad_bnb"] += t_b * cnt
            if a.fp8 and "fp8_dgrad_us" in r:
                t8b = timeit(lambda: igemm_dgrad(dy, wt8, (H, H), s, p, k, k, bnb=bnb, fp8=f8d))
                line += f" | fp8 dgrad+bnb {t8b:8.1f}"
                r["fp8_dgrad_bnb_us"] = t8b
                tot["fp8_dgrad_bnb"] += t8b * cnt
        if a.tiles and not stem:
            yref = igemm_fwd(x, w, s, p, k, k).float()
            dref = igemm_dgrad(dy, wt, (H, H), s, p, k, k).float()

            def rel(u, v):
                return float((u.float() - v).norm() / v.norm().clamp_min(1e-30))
            for t in (int(v) for v in a.tiles.split(",")):
                # fwd and dgrad separately: a tile may cover one direction only (n/a = -1)
                tf = td = ef = ed = -1.0
                try:
                    ef = rel(igemm_fwd(x, w, s, p, k, k, tile=t), yref)
                    tf = timeit(lambda: igemm_fwd(x, w, s, p, k, k, stats=stats, tile=t))
                except RuntimeError:
                    pass
                try:
                    ed = rel(igemm_dgrad(dy, wt, (H, H), s, p, k, k, tile=t), dref)
                    td = timeit(lambda: igemm_dgrad(dy, wt, (H, H), s, p, k, k, tile=t))
                except RuntimeError:
                    pass
                if tf < 0 and td < 0:  # a tile that does not cover this shape
                    line += f"\n      tile {t}: n/a"
                    continue
                line += f"\n      tile {t}: fwd {tf:8.1f} us {flops / max(tf, 1e-9) / 1e6:6.0f} TF | dgrad {td:8.1f} us " \
                        f"{flops / max(td, 1e-9) / 1e6:6.0f} TF | rel err vs auto fwd {ef:.1e} dgrad {ed:.1e}"
                if bnb is not None:
                    try:
                        tb = timeit(lambda: igemm_dgrad(dy, wt, (H, H), s, p, k, k, bnb=bnb, tile=t))
                        line += f" | dgrad+bnb {tb:8.1f}"
                    except RuntimeError:
                        line += " | dgrad+bnb n/a"
                r[f"tile{t}"] = (tf, td, ef, ed)
                if ef > 2e-2 or ed > 2e-2:
                    line += "  <-- MISMATCH"
                tot[f"tile{t}_fwd"] += max(tf, 0.0) * cnt
                tot[f"tile{t}_dgrad"] += max(td, 0.0) * cnt
        print(line, flush=True)
        rows.append(r)
        tot["fwd"] += t_f * cnt
        tot["dgrad"] += t_d * cnt
        tot["wgrad"] += t_w * cnt
        tot["miopen"] += r.get("miopen_fwd_us", 0) * cnt
    print("totals (us, per step):", {k: round(v, 1) for k, v in tot.items()})
    if a.json:
        json.dump(dict(rows=rows, totals=tot), open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
