"""Every unique ResNet-50 (224²) and ResNet-18 (448²) conv shape at the bench's
per-GPU batch, through the AUTO-dispatched kernels, against fp32 PyTorch.

VERDICT r1 weak #4: the dispatcher picks the 256x256 LDS-DMA tiles, persistent
grids, the streaming short-K kernel and split-K wgrads by problem size, so toy
shapes do not exercise what the bench runs. Here each shape runs at the batch
the bench uses (R50: 1024 per GPU; R18@448: 128, the reference's batch,
imagenet.py:442) -- forward with BN statistics, dgrad plain and with the fused
BN-backward epilogue (IG_BNBWD, as the model's blocks issue it), wgrad -- and
the kernel names the auto-dispatch launched are recorded with torch.profiler
(``gpurun_out/conv_shape_kernels.json``, committed as
``profiles/conv_shape_kernels.md``); the set over all shapes must cover the
conv kernels of the bench's rocprof trace (``BENCH_KERNELS``, from
``profiles/r50_b1024_v21_stream_tables.md``).
Reference ops: torchvision resnet convs (imagenet.py:312, fwd :123, bwd :128).
"""

import collections
import json
import os
import sys

import pytest
import torch
import torch.nn.functional as F

pytestmark = [pytest.mark.gpu, pytest.mark.slow]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
DEV = "cuda"
KERNELS = collections.OrderedDict()


def _shapes(arch, size, batch):
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    from conv_bench import shapes
    return [(batch,) + k for k in shapes(arch, batch, size)]


SHAPES = _shapes("resnet50", 224, 1024) + [(1024, 2048, 1, 1000, 1, 1, 0)] + _shapes("resnet18", 448, 128)

# conv kernel templates in the R50 bench trace (round 5 HEAD, profiles/r50_b1024_r5_standalone.md: v3 with its
# element-size / format template arguments, the streaming kernel with its second-K-segment width); update together
# with the dispatcher. Not listed (no plain conv shape takes them; tests/test_model_gpu.py covers them against the
# fp32 model in test_bn_gram_backward_matches_torch and test_fp8_forward_training_step[resnet50-gram]): the
# fused-output conv3 mode conv_stream_kernel<*, *, *, 4, ...> (bn3 + shortcut + ReLU + mask bits / e4m3 copy) and
# the Gram-form bn3 dgrad over [g | h2], conv_stream_kernel<256, 64, 2, 2, false, false, 64>, and the stem weight
# gradient with the stem BN's backward apply fused in, stem_wgrad_band_kernel<2, true> (ops.misc.StemFn,
# test_model_gpu.py::test_stem_fn_matches_unfused).
BENCH_KERNELS = [
    "conv_stream_kernel<128, 128, 2, 1, false, false, 0>",
    "conv_stream_kernel<128, 128, 2, 3, false, false, 0>",
    "conv_stream_kernel<256, 128, 2, 1, false, false, 0>",
    "conv_stream_kernel<256, 64, 2, 0, false, false, 0>",
    "conv_stream_kernel<256, 64, 2, 1, false, false, 0>",
    "conv_stream_kernel<256, 64, 2, 3, false, false, 0>",
    "conv_stream_kernel<64, 128, 3, 1, false, false, 0>",
    "conv_stream_kernel<64, 128, 3, 3, false, false, 0>",
    "conv_stream_kernel<64, 256, 3, 0, false, false, 0>",
    "conv_stream_kernel<64, 64, 3, 0, false, false, 0>",
    "halo3x3_kernel<56, 4, 0>",
    "halo3x3_kernel<56, 4, 1>",
    "igemm_dma_kernel<128, 128, 2, 2, 0, 4, 0, 2, 0, 128>",
    "igemm_dma_kernel<128, 128, 2, 2, 1, 4, 2, 2, 0, 128>",
    "igemm_v3_kernel<128, 128, 2, 2, 4, 128, 2, 0, false>",
    "igemm_v3_kernel<256, 256, 2, 2, 8, 128, 2, 0, false>",
    "stem_band_kernel<4>",
    "wgrad_halo_kernel<14, 14, 7, 16>",
    "wgrad_halo_kernel<28, 4, 4, 32>",
    "wgrad_halo_kernel<56, 4, 7, 64>",
    "wgrad_kernel<128, 128, 2, false, 4, 32, false>",
    "wgrad_kernel<128, 128, 2, false, 4, 64, false>",
    "wgrad_kernel<64, 128, 1, false, 4, 32, false>",
    "stem_wgrad_band_kernel<4, false>",
    "wgrad_v3_kernel<64, 2, 2, 2, 0>",
]


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


def _kernels(fn):
    """Run fn under torch.profiler; the GPU kernel names it launched."""
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        out = fn()
        torch.cuda.synchronize()
    names = [e.name for e in prof.events() if e.device_type.name == "CUDA"]
    return out, [n for n in names if any(k in n for k in ("igemm", "conv_stream", "wgrad_", "halo3x3", "stem_band"))]


def _short(names):
    return sorted({n.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0] for n in names})


@pytest.mark.parametrize("shape", SHAPES, ids=[f"N{s[0]}_C{s[1]}_H{s[2]}_K{s[3]}_k{s[4]}s{s[5]}" for s in SHAPES])
def test_production_conv_shape(shape):
    from imagent_amd.models.resnet import BatchNorm2d, BNWork
    from imagent_amd.ops import _lib
    from imagent_amd.ops.bn import relu_mask_bits
    from imagent_amd.ops.conv import BNBwdFuse, igemm_dgrad, igemm_fwd, igemm_wgrad
    N, Ci, H, Co, k, s, p = shape
    stem = Ci == 3
    torch.manual_seed(0)
    Cx = 4 if stem else Ci
    x = torch.randn(N, H, H, Cx, device=DEV).to(torch.bfloat16)
    if stem:
        x[..., 3] = 0
    w = (torch.randn(Co, k, k, Ci, device=DEV) * (2.0 / (Ci * k * k)) ** 0.5).to(torch.bfloat16)
    # fwd / dgrad are per image: the fp32 reference runs on the first two and the last two
    # images (a wave-quantisation tail split runs the last images through another kernel)
    SEL = torch.tensor([0, 1, N - 2, N - 1], device=DEV)
    NS = len(SEL)
    xr = x[SEL][..., :Ci].permute(0, 3, 1, 2).float()
    wr = w.permute(0, 3, 1, 2).float()
    OH = (H + 2 * p - k) // s + 1
    rec = {}

    # ---- forward + BN statistics (slab: raw sums, shift 0)
    slab = torch.zeros(_lib.STAT_SLOTS, 2, Co, device=DEV)
    if stem:
        wrow = torch.zeros(Co, k, 32, dtype=torch.bfloat16, device=DEV)
        wrow[:, :, :k * 4].view(Co, k, k, 4)[..., :3] = w
        y, rec["fwd"] = _kernels(lambda: igemm_fwd(x, wrow, s, p, k, k, stats=slab, stem=True))
    else:
        y, rec["fwd"] = _kernels(lambda: igemm_fwd(x, w, s, p, k, k, stats=slab))
    ref = F.conv2d(xr, wr, None, s, p)
    assert tuple(y.shape) == (N, OH, OH, Co)
    assert rel(y[SEL].permute(0, 3, 1, 2), ref) < 1e-2
    yf = y.float().reshape(-1, Co)
    tot = slab.sum(0)
    assert rel(tot[0], yf.sum(0)) < 1e-3 and rel(tot[1], (yf * yf).sum(0)) < 1e-3
    del ref

    g = torch.randn(N, OH, OH, Co, device=DEV).to(torch.bfloat16)
    gr = g[SEL].permute(0, 3, 1, 2).float()
    if not stem:
        # ---- dgrad (plain)
        wt = w.permute(3, 1, 2, 0).contiguous()  # [Ci][KH][KW][Co]
        dx, rec["dgrad"] = _kernels(lambda: igemm_dgrad(g, wt, (H, H), s, p, k, k))
        dref = torch.nn.grad.conv2d_input((NS, Ci, H, H), wr, gr, s, p)
        assert rel(dx[SEL].permute(0, 3, 1, 2), dref) < 1e-2
        # ---- dgrad with the fused BN-backward epilogue (mask recomputed from the BN input)
        if Ci % 8 == 0 and k >= s:  # (the model never fuses into a strided 1x1 dgrad)
            bn = BatchNorm2d(Ci).to(DEV)
            with torch.no_grad():
                bn.weight.uniform_(0.5, 1.5)
                bn.bias.uniform_(-0.5, 0.5)
            xb = torch.randn(N, H, H, Ci, device=DEV).to(torch.bfloat16)
            mean = xb.float().reshape(-1, Ci).mean(0)
            rstd = torch.rsqrt(xb.float().reshape(-1, Ci).var(0, unbiased=False) + 1e-5)
            save = torch.stack([mean, rstd])
            bn.work = BNWork(torch.zeros(_lib.STAT_SLOTS, 2, Ci, device=DEV), torch.zeros(2, Ci, device=DEV),
                             save, torch.zeros(_lib.kernels().imk_bn_bwd_scratch_floats(Ci), device=DEV))
            db, rec["dgrad_bnb"] = _kernels(lambda: igemm_dgrad(g, wt, (H, H), s, p, k, k,
                                                               bnb=BNBwdFuse(xb, bn)))
            xhat = (xb.float() - mean) * rstd
            keep = (xhat * bn.weight.detach() + bn.bias.detach()) > 0
            gm = dref.permute(0, 2, 3, 1) * keep[SEL]
            assert rel(db[SEL], gm) < 1e-2
            sl = bn.work.scratch[: _lib.STAT_SLOTS * 3 * Ci].view(_lib.STAT_SLOTS, 3, Ci).sum(0)
            gmb = db.float()
            assert rel(sl[0], (gmb * xhat).reshape(-1, Ci).sum(0)) < 2e-3
            assert rel(sl[1], gmb.reshape(-1, Ci).sum(0)) < 2e-3
            # ReLU mask from a saved output y (BN + residual + ReLU: the blocks' last BN)
            yb = torch.relu(torch.randn(N, H, H, Ci, device=DEV)).to(torch.bfloat16)
            bn.work.scratch.zero_()
            dy_, rec["dgrad_bnb_y"] = _kernels(lambda: igemm_dgrad(g, wt, (H, H), s, p, k, k,
                                                                  bnb=BNBwdFuse(xb, bn, y=relu_mask_bits(yb))))
            assert rel(dy_[SEL], dref.permute(0, 2, 3, 1) * (yb[SEL] > 0)) < 1e-2
            if k == 1 and s == 1:
                # + the downsample BN branch (mode 2: the previous block's last BN pair)
                bn2 = BatchNorm2d(Ci).to(DEV)
                x2 = torch.randn(N, H, H, Ci, device=DEV).to(torch.bfloat16)
                m2 = x2.float().reshape(-1, Ci).mean(0)
                r2 = torch.rsqrt(x2.float().reshape(-1, Ci).var(0, unbiased=False) + 1e-5)
                bn2.work = BNWork(None, None, torch.stack([m2, r2]), None)
                bn.work.scratch.zero_()
                d2, rec["dgrad_bnb_y_x2"] = _kernels(lambda: igemm_dgrad(
                    g, wt, (H, H), s, p, k, k, bnb=BNBwdFuse(xb, bn, y=relu_mask_bits(yb), x2=x2, bn2=bn2)))
                assert rel(d2[SEL], dref.permute(0, 2, 3, 1) * (yb[SEL] > 0)) < 1e-2
                sl = bn.work.scratch[: _lib.STAT_SLOTS * 3 * Ci].view(_lib.STAT_SLOTS, 3, Ci).sum(0)
                x2hat = (x2.float() - m2) * r2
                assert rel(sl[2], (d2.float() * x2hat).reshape(-1, Ci).sum(0)) < 2e-3
        del dref
    # ---- wgrad (fp32 accumulation into the arena slot)
    if stem:
        dw = torch.zeros(Co, k, 32, device=DEV)
        _, rec["wgrad"] = _kernels(lambda: igemm_wgrad(g, x, dw, s, p, k, k, stem=True))
        got = dw[:, :, :k * 4].view(Co, k, k, 4)[..., :3]
    else:
        dw = torch.zeros(Co, k * k * Ci, device=DEV)
        _, rec["wgrad"] = _kernels(lambda: igemm_wgrad(g, x, dw, s, p, k, k))
        got = dw.view(Co, k, k, Ci)
    # the weight gradient sums over ALL images: fp32 reference over the full batch
    wref = torch.nn.grad.conv2d_weight(x[..., :Ci].permute(0, 3, 1, 2).float(), (Co, Ci, k, k),
                                       g.permute(0, 3, 1, 2).float(), s, p)
    assert rel(got.permute(0, 3, 1, 2), wref) < 1e-2

    if s == 1 and ((k == 1 and Ci in (64, 128) and Co % 128 == 0) or
                   (k == 3 and Ci == Co == 64 and H in (56, 112))):
        # ---- BN apply + ReLU on the operand path (IMAGENT_BN_XFUSE: bottleneck conv3's of stages 1-2, the
        # halo-tiled 64 -> 64 3x3 convs)
        ss = torch.stack([torch.rand(Ci, device=DEV) + 0.5, torch.randn(Ci, device=DEV) * 0.3]).contiguous()
        hx = torch.relu(x.float() * ss[0] + ss[1]).to(torch.bfloat16)
        yx, rec["fwd_xbn"] = _kernels(lambda: igemm_fwd(x, w, 1, p, k, k, stats=slab, xbn=ss))
        assert rel(yx[SEL].permute(0, 3, 1, 2), F.conv2d(hx[SEL].permute(0, 3, 1, 2).float(), wr, None, 1, p)) < 1e-2
        dwx = torch.zeros(Co, k * k * Ci, device=DEV)
        _, rec["wgrad_xbn"] = _kernels(lambda: igemm_wgrad(g, x, dwx, 1, p, k, k, xbn=ss))
        wxr = torch.nn.grad.conv2d_weight(hx.permute(0, 3, 1, 2).float(), (Co, Ci, k, k),
                                          g.permute(0, 3, 1, 2).float(), 1, p)
        assert rel(dwx.view(Co, k, k, Ci).permute(0, 3, 1, 2), wxr) < 1e-2

    for op, names in rec.items():
        assert names, f"{op}: the profiler saw no conv kernel (auto-dispatch launched nothing?)"
        KERNELS[f"{shape} {op}"] = _short(names)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "conv_shape_kernels.json"), "w") as f:
        json.dump(KERNELS, f, indent=1)


def test_variants_cover_the_bench_trace():
    """Run after the shape tests: every conv kernel template the R50 bench launches
    was exercised above (by the auto-dispatch, on production shapes)."""
    if not KERNELS:
        pytest.skip("shape tests did not run in this session")
    seen = {n for v in KERNELS.values() for n in v}
    missing = sorted(b for b in BENCH_KERNELS if b not in seen)
    assert not missing, f"bench kernels not covered by the shape tests: {missing}; seen {sorted(seen)}"
