"""Numerics of every HIP kernel vs a plain-PyTorch fp32 reference of the same op.

Inputs are bf16-rounded first, the reference runs in fp32 on those values,
and the comparison is a relative L2 error sized for bf16 outputs.
"""

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def rel(a, b):
    a = a.float()
    b = b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


def bf(t):
    return t.to(torch.bfloat16)


def nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


def nchw(t):
    return t.permute(0, 3, 1, 2).contiguous()


CONV_SHAPES = [
    # N, Ci, H, Co, k, s, p
    (4, 64, 14, 64, 1, 1, 0),
    (4, 64, 14, 128, 3, 1, 1),
    (4, 128, 14, 64, 3, 2, 1),
    (2, 256, 9, 512, 1, 2, 0),
    (2, 8, 32, 64, 7, 2, 3),      # stem (padded channels)
    (3, 72, 11, 200, 3, 1, 1),    # ragged M / N / K tails
    (2, 2048, 1, 1000, 1, 1, 0),  # fc as 1x1 conv
]


@pytest.mark.parametrize("shape", CONV_SHAPES)
def test_conv_fwd_dgrad_wgrad(shape):
    from imagent_amd.ops.conv import igemm_dgrad, igemm_fwd, igemm_wgrad
    N, Ci, H, Co, k, s, p = shape
    torch.manual_seed(0)
    x = bf(torch.randn(N, Ci, H, H, device=DEV))
    w = bf(torch.randn(Co, Ci, k, k, device=DEV) * (2.0 / (Ci * k * k)) ** 0.5)
    xr = x.float().requires_grad_(True)
    wr = w.float().requires_grad_(True)
    yr = F.conv2d(xr, wr, None, s, p)
    g = bf(torch.randn_like(yr))
    yr.backward(g.float())

    slab = torch.zeros(32, 2, Co, device=DEV)
    y = igemm_fwd(nhwc(x), nhwc(w), s, p, k, k, stats=slab)
    stats = slab.sum(0)
    assert rel(nchw(y), yr) < 1e-2
    # epilogue BN statistics of the bf16 output
    yb = nchw(y).float()
    assert rel(stats[0], yb.sum((0, 2, 3))) < 1e-3
    assert rel(stats[1], (yb * yb).sum((0, 2, 3))) < 1e-3

    wt = w.permute(1, 2, 3, 0).contiguous()  # [Ci][KH][KW][Co]
    dx = igemm_dgrad(nhwc(g), wt, (H, H), s, p, k, k)
    assert rel(nchw(dx), xr.grad) < 1e-2

    dw = torch.zeros(Co, k, k, Ci, device=DEV)
    igemm_wgrad(nhwc(g), nhwc(x), dw, s, p, k, k)
    assert rel(dw.permute(0, 3, 1, 2), wr.grad) < 5e-3
    # accumulation semantics (+=)
    igemm_wgrad(nhwc(g), nhwc(x), dw, s, p, k, k)
    assert rel(dw.permute(0, 3, 1, 2), 2 * wr.grad) < 5e-3


@pytest.mark.parametrize("tile", [1, 2, 3, 4, 5, 6, 7, 8, 9])
@pytest.mark.parametrize("shape", [(4, 64, 14, 128, 3, 1, 1), (3, 72, 11, 200, 3, 2, 1), (2, 256, 9, 320, 1, 1, 0)])
def test_conv_explicit_tiles(tile, shape):
    """Every main-loop / tile variant the dispatcher can pick, incl. ragged tails."""
    from imagent_amd.ops.conv import igemm_dgrad, igemm_fwd
    N, Ci, H, Co, k, s, p = shape
    torch.manual_seed(1)
    x = bf(torch.randn(N, Ci, H, H, device=DEV))
    w = bf(torch.randn(Co, Ci, k, k, device=DEV) * (2.0 / (Ci * k * k)) ** 0.5)
    xr = x.float().requires_grad_(True)
    yr = F.conv2d(xr, w.float(), None, s, p)
    g = bf(torch.randn_like(yr))
    yr.backward(g.float())
    slab = torch.zeros(32, 2, Co, device=DEV)
    y = igemm_fwd(nhwc(x), nhwc(w), s, p, k, k, stats=slab, tile=tile)
    assert rel(nchw(y), yr) < 1e-2
    yb = nchw(y).float()
    assert rel(slab.sum(0)[0], yb.sum((0, 2, 3))) < 1e-3
    dx = igemm_dgrad(nhwc(g), w.permute(1, 2, 3, 0).contiguous(), (H, H), s, p, k, k, tile=tile)
    assert rel(nchw(dx), xr.grad) < 1e-2


@pytest.mark.parametrize("tile", [0, 2, 4, 8])
@pytest.mark.parametrize("shape", [(4, 64, 14, 128, 3, 1, 1), (3, 72, 11, 200, 3, 2, 1), (2, 256, 9, 512, 1, 1, 0),
                                   (5, 96, 7, 64, 1, 1, 0), (2, 64, 8, 256, 1, 1, 0), (3, 128, 15, 320, 3, 1, 1)])
def test_conv_lds_epilogue(tile, shape):
    """LDS-staged coalesced epilogue: forward + statistics, dgrad, dgrad accumulate
    (ragged M / N / K)."""
    from imagent_amd.ops.conv import igemm_dgrad, igemm_fwd
    N, Ci, H, Co, k, s, p = shape
    torch.manual_seed(4)
    x = bf(torch.randn(N, Ci, H, H, device=DEV))
    w = bf(torch.randn(Co, Ci, k, k, device=DEV) * (2.0 / (Ci * k * k)) ** 0.5)
    xr = x.float().requires_grad_(True)
    yr = F.conv2d(xr, w.float(), None, s, p)
    g = bf(torch.randn_like(yr))
    yr.backward(g.float())
    slab = torch.zeros(32, 2, Co, device=DEV)
    y = igemm_fwd(nhwc(x), nhwc(w), s, p, k, k, stats=slab, tile=tile, epi=2)
    assert rel(nchw(y), yr) < 1e-2
    yb = nchw(y).float()
    assert rel(slab.sum(0)[0], yb.sum((0, 2, 3))) < 1e-3
    assert rel(slab.sum(0)[1], (yb * yb).sum((0, 2, 3))) < 1e-3
    wt = w.permute(1, 2, 3, 0).contiguous()
    dx = igemm_dgrad(nhwc(g), wt, (H, H), s, p, k, k, tile=tile, epi=2)
    assert rel(nchw(dx), xr.grad) < 1e-2
    base = bf(torch.randn(N, H, H, Ci, device=DEV))
    acc = base.clone()
    igemm_dgrad(nhwc(g), wt, (H, H), s, p, k, k, out=acc, accumulate=True, tile=tile, epi=2)
    assert rel(acc.float() - base.float(), nhwc(xr.grad)) < 2e-2


@pytest.mark.parametrize("tile", [17, 18, 19])
@pytest.mark.parametrize("shape", [(4, 64, 14, 128, 3, 1, 1), (2, 256, 9, 512, 1, 1, 0), (2, 64, 8, 256, 1, 1, 0),
                                   (3, 128, 15, 320, 3, 1, 1), (3, 128, 15, 320, 3, 2, 1), (8, 256, 14, 256, 3, 1, 1),
                                   (2, 128, 9, 192, 1, 1, 0), (3, 64, 5, 192, 3, 2, 1), (2, 512, 7, 2048, 1, 1, 0)])
def test_conv_v3(tile, shape):
    """v3 main loop (conv_igemm_v3.h; 17: 256x256, 18: 128x128, 19: 256x128): buffer-descriptor LDS-DMA whose
    out-of-image taps / rows beyond M or Nout read the buffer unit's zeros -- padding borders,
    strided dgrad parity classes (taps with negative offsets), ragged M and N -- forward +
    statistics, dgrad, dgrad accumulate against fp32; 1 to 36 K-tiles."""
    test_conv_lds_epilogue(tile, shape)


@pytest.mark.parametrize("shape", [(4, 64, 14, 256, 1), (3, 64, 9, 128, 1), (2, 128, 11, 512, 1), (5, 128, 7, 128, 1),
                                   (3, 64, 56, 64, 3), (2, 64, 112, 64, 3)])
def test_conv_xbn_operand(shape):
    """BatchNorm apply + ReLU on the operand path (IMAGENT_BN_XFUSE): the streaming 1x1 forward
    (with statistics) and the weight gradient take the BN INPUT x and a per-channel (scale, shift),
    against fp32 convs of relu(x * scale + shift) rounded to bf16 (what the BN pass would store);
    negative scales, ragged pixel counts."""
    from imagent_amd.ops.conv import igemm_fwd, igemm_wgrad
    N, Ci, H, Co, k = shape  # k = 3: the halo-tiled 64 -> 64 kernel (zero padding must stay 0)
    p = k // 2
    torch.manual_seed(11)
    x = bf(torch.randn(N, H, H, Ci, device=DEV) * 2 + 0.5)
    ss = torch.stack([torch.randn(Ci, device=DEV), torch.randn(Ci, device=DEV) * 0.5]).contiguous()
    h = torch.relu(x.float() * ss[0] + ss[1]).to(torch.bfloat16).float()  # [N, H, W, Ci]
    w = bf(torch.randn(Co, k, k, Ci, device=DEV) * (2.0 / (Ci * k * k)) ** 0.5)
    wr = w.float().permute(0, 3, 1, 2)
    ref = F.conv2d(h.permute(0, 3, 1, 2), wr, None, 1, p)  # NCHW
    slab = torch.zeros(32, 2, Co, device=DEV)
    y = igemm_fwd(x, w, 1, p, k, k, stats=slab, xbn=ss)
    assert rel(y.permute(0, 3, 1, 2), ref) < 1e-2
    yb = y.float()
    assert rel(slab.sum(0)[0], yb.sum((0, 1, 2))) < 1e-3
    assert rel(slab.sum(0)[1], (yb * yb).sum((0, 1, 2))) < 1e-3
    g = bf(torch.randn(N, H, H, Co, device=DEV))
    dw = torch.zeros(Co, k * k * Ci, device=DEV)
    igemm_wgrad(g, x, dw, 1, p, k, k, xbn=ss)
    wref = torch.nn.grad.conv2d_weight(h.permute(0, 3, 1, 2), (Co, Ci, k, k), g.float().permute(0, 3, 1, 2), 1, p)
    assert rel(dw.view(Co, k, k, Ci).permute(0, 3, 1, 2), wref) < 1e-2


@pytest.mark.parametrize("splits", [0, 3])
@pytest.mark.parametrize("shape", [(4, 64, 14, 128, 3, 1, 1), (3, 72, 11, 200, 3, 2, 1), (2, 256, 9, 512, 1, 2, 0),
                                   (2, 128, 7, 256, 3, 1, 1), (5, 96, 13, 136, 1, 1, 0)])
def test_wgrad_variants(shape, splits):
    """Weight gradient incl. ragged Co / K tails and explicit split-K."""
    from imagent_amd.ops.conv import igemm_wgrad
    N, Ci, H, Co, k, s, p = shape
    torch.manual_seed(6)
    x = bf(torch.randn(N, Ci, H, H, device=DEV))
    w = torch.randn(Co, Ci, k, k, device=DEV).requires_grad_(True)
    yr = F.conv2d(x.float(), w, None, s, p)
    g = bf(torch.randn_like(yr))
    yr.backward(g.float())
    dw = torch.zeros(Co, k, k, Ci, device=DEV)
    igemm_wgrad(nhwc(g), nhwc(x), dw, s, p, k, k, splits=splits)
    assert rel(dw.permute(0, 3, 1, 2), w.grad) < 5e-3


@pytest.mark.parametrize("variant", [-1, 1, 2, 3, 4])
@pytest.mark.parametrize("shape", [(4, 128, 14, 128, 3, 1, 1), (3, 256, 9, 128, 3, 2, 1), (2, 128, 7, 256, 3, 1, 1),
                                   (3, 256, 11, 384, 1, 1, 0), (2, 128, 10, 256, 1, 2, 0), (1, 128, 5, 128, 3, 1, 1),
                                   (3, 64, 13, 256, 1, 1, 0), (2, 64, 10, 128, 1, 2, 0), (3, 256, 9, 64, 1, 1, 0),
                                   (2, 64, 11, 64, 1, 1, 0)])
def test_wgrad_v3(shape, variant):
    """LDS-DMA weight gradient (conv_wgrad_v3.h, Ci and Co % 128 == 0, or 64 on a 1x1) and the
    register-staged kernel on the same shapes: 3x3 stride 1 / 2 with image borders, 1x1 dense and strided
    (Ci = 64: one half-used k tile), an M that is not a multiple of the stage rows, explicit split-K."""
    from imagent_amd.ops.conv import igemm_wgrad
    N, Ci, H, Co, k, s, p = shape
    torch.manual_seed(7)
    x = bf(torch.randn(N, Ci, H, H, device=DEV))
    w = torch.randn(Co, Ci, k, k, device=DEV).requires_grad_(True)
    yr = F.conv2d(x.float(), w, None, s, p)
    g = bf(torch.randn_like(yr))
    yr.backward(g.float())
    for splits in (0, 3):
        dw = torch.zeros(Co, k, k, Ci, device=DEV)
        igemm_wgrad(nhwc(g), nhwc(x), dw, s, p, k, k, splits=splits, variant=variant)
        assert rel(dw.permute(0, 3, 1, 2), w.grad) < 5e-3, splits


@pytest.mark.parametrize("p", [64, 128, 256])
@pytest.mark.parametrize("M", [4096 * 3 + 2, 2048 * 56 * 7, 999])
def test_gram_sym(p, M):
    """The Gram-form bottleneck's G += h2^T h2 (ops/bn_gram.py gram_G): one staged operand read as both fragments
    (p = 128), pixel pairs whose diagonal quadrants sum to G (p = 64), the plain weight gradient otherwise / for odd M;
    against fp32, and accumulating into G."""
    from imagent_amd.ops.bn_gram import gram_G
    torch.manual_seed(3)
    h2 = bf(torch.randn(M, 1, 1, p, device=DEV) + 0.5)  # (NHWC, as the model holds it)
    ref = h2.view(M, p).float().t() @ h2.view(M, p).float()
    G = torch.ones(p, p, device=DEV)
    gram_G(h2, G)
    assert rel(G - 1.0, ref) < 2e-4  # (fp32 sums over up to 8e5 rows in two different orders)


@pytest.mark.parametrize("N", [3, 12])
def test_stem_wgrad_band(N):
    """The 7x7 / stride-2 stem's band weight gradient (conv_wgrad_stem.h: dY and the input rows of a band staged in
    LDS, both operands by transposing reads, per-block accumulators) against the fp32 conv weight gradient and the
    register-staged stem kernel (variant -2); N = 12 gives 672 bands, more than one per resident block."""
    from imagent_amd.ops.conv import igemm_wgrad
    torch.manual_seed(5)
    x = torch.zeros(N, 224, 224, 4, device=DEV)
    x[..., :3] = torch.randn(N, 224, 224, 3, device=DEV)
    x = bf(x)
    w = torch.randn(64, 4, 7, 7, device=DEV).requires_grad_(True)
    yr = F.conv2d(nchw(x).float(), w, None, 2, 3)
    g = bf(torch.randn_like(yr))
    yr.backward(g.float())
    ref = w.grad.permute(0, 2, 3, 1)  # [co][kh][kw][ci]
    for variant in (0, -2):
        dw = torch.zeros(64, 7, 32, device=DEV)
        igemm_wgrad(nhwc(g), x, dw, 2, 3, 7, 7, stem=True, variant=variant)
        got = dw[:, :, :28].reshape(64, 7, 7, 4)
        assert rel(got, ref) < 5e-3, variant


@pytest.mark.parametrize("variant", [6])
@pytest.mark.parametrize("shape", [(3, 256, 11, 256, 1, 1, 0), (2, 256, 10, 512, 1, 2, 0), (2, 512, 7, 256, 3, 1, 1),
                                   (2, 256, 9, 768, 1, 1, 0), (1, 256, 5, 512, 3, 2, 1)])
def test_wgrad_v3_wide(shape, variant):
    """The wide wgrad_v3 tile (256 x 256 on 16 waves, one block per CU, staged as 128-channel sub-images) against
    the fp32 conv weight gradient; 1x1 dense / strided and 3x3 with borders, ragged M, explicit split-K."""
    from imagent_amd.ops.conv import igemm_wgrad
    N, Ci, H, Co, k, s, p = shape
    torch.manual_seed(7)
    x = bf(torch.randn(N, Ci, H, H, device=DEV))
    w = torch.randn(Co, Ci, k, k, device=DEV).requires_grad_(True)
    yr = F.conv2d(x.float(), w, None, s, p)
    g = bf(torch.randn_like(yr))
    yr.backward(g.float())
    for splits in (0, 3):
        dw = torch.zeros(Co, k, k, Ci, device=DEV)
        igemm_wgrad(nhwc(g), nhwc(x), dw, s, p, k, k, splits=splits, variant=variant)
        assert rel(dw.permute(0, 3, 1, 2), w.grad) < 5e-3, splits


@pytest.mark.parametrize("N,Ci,Co,H,W", [(3, 64, 64, 56, 56), (5, 64, 64, 8, 56), (1, 64, 64, 4, 56),
                                         (3, 128, 128, 28, 28), (2, 64, 192, 8, 28), (2, 256, 256, 14, 14),
                                         (3, 128, 64, 14, 14), (3, 512, 512, 7, 7), (1, 64, 128, 7, 7)])
def test_wgrad_halo(N, Ci, Co, H, W):
    """Halo-tiled 3x3 weight gradient (conv_wgrad_halo.h, variant 9) against the fp32 conv weight gradient:
    64-channel co / ci slices, image borders on every side, bands crossing images, zero-padded k rows
    (W 28 / 14 / 7), more ranges than bands; the default dispatch picks it; += semantics."""
    from imagent_amd.ops.conv import igemm_wgrad
    torch.manual_seed(11)
    x = bf(torch.randn(N, Ci, H, W, device=DEV))
    w = torch.randn(Co, Ci, 3, 3, device=DEV).requires_grad_(True)
    yr = F.conv2d(x.float(), w, None, 1, 1)
    g = bf(torch.randn_like(yr))
    yr.backward(g.float())
    for variant in (9, 0):  # (the default dispatch keeps W 7 on the register-staged kernel)
        dw = torch.zeros(Co, 3, 3, Ci, device=DEV)
        igemm_wgrad(nhwc(g), nhwc(x), dw, 1, 1, 3, 3, variant=variant)
        assert rel(dw.permute(0, 3, 1, 2), w.grad) < 5e-3, variant
    dw0 = torch.ones(Co, 3, 3, Ci, device=DEV)  # accumulates (+=) into the gradient
    igemm_wgrad(nhwc(g), nhwc(x), dw0, 1, 1, 3, 3, variant=9)
    assert rel(dw0.permute(0, 3, 1, 2) - 1.0, w.grad) < 5e-3


@pytest.mark.parametrize("N,Ci,Co,H,W", [(3, 128, 128, 56, 56), (2, 64, 192, 8, 56), (1, 64, 64, 4, 56),
                                         (2, 256, 256, 28, 28), (3, 128, 64, 4, 28), (3, 512, 512, 14, 14),
                                         (1, 64, 128, 14, 14)])
def test_wgrad_stride2(N, Ci, Co, H, W):
    """Stride-2 3x3 weight gradients (the bottlenecks' strided conv2) against the fp32 conv weight gradient, through
    the default dispatch and the register-staged kernel: output widths 28 / 14 / 7, top / left padding taps,
    ragged M; +=. (The halo-tiled kernel takes stride 1 only: its stride-2 phase-plane form measured slower and
    was removed in round 5.)"""
    from imagent_amd.ops.conv import igemm_wgrad
    torch.manual_seed(12)
    x = bf(torch.randn(N, Ci, H, W, device=DEV))
    w = torch.randn(Co, Ci, 3, 3, device=DEV).requires_grad_(True)
    yr = F.conv2d(x.float(), w, None, 2, 1)
    g = bf(torch.randn_like(yr))
    yr.backward(g.float())
    for variant in (0, -1):
        dw = torch.zeros(Co, 3, 3, Ci, device=DEV)
        igemm_wgrad(nhwc(g), nhwc(x), dw, 2, 1, 3, 3, variant=variant)
        assert rel(dw.permute(0, 3, 1, 2), w.grad) < 5e-3, variant
    dw0 = torch.ones(Co, 3, 3, Ci, device=DEV)
    igemm_wgrad(nhwc(g), nhwc(x), dw0, 2, 1, 3, 3)
    assert rel(dw0.permute(0, 3, 1, 2) - 1.0, w.grad) < 5e-3


def test_stem_row_segment_conv():
    """7x7/s2 stem: 4-channel NHWC input, [Co][KH][32] weight rows (fwd + wgrad)."""
    from imagent_amd.ops.conv import igemm_fwd, igemm_wgrad
    torch.manual_seed(7)
    N, H, Co = 3, 38, 64
    x3 = bf(torch.randn(N, 3, H, H, device=DEV))
    w3 = bf(torch.randn(Co, 3, 7, 7, device=DEV) * 0.1)
    xr = x3.float().requires_grad_(True)
    wr = w3.float().requires_grad_(True)
    yr = F.conv2d(xr, wr, None, 2, 3)
    g = bf(torch.randn_like(yr))
    yr.backward(g.float())
    x4 = torch.zeros(N, H, H, 4, device=DEV, dtype=torch.bfloat16)
    x4[..., :3] = nhwc(x3)
    wrow = torch.zeros(Co, 7, 32, device=DEV, dtype=torch.bfloat16)
    wrow[:, :, :28].view(Co, 7, 7, 4)[..., :3] = w3.permute(0, 2, 3, 1)
    slab = torch.zeros(32, 2, Co, device=DEV)
    y = igemm_fwd(x4, wrow, 2, 3, 7, 7, stats=slab, stem=True)
    stats = slab.sum(0)
    assert rel(nchw(y), yr) < 1e-2
    assert rel(stats[0], nchw(y).float().sum((0, 2, 3))) < 1e-3
    dw = torch.zeros(Co, 7, 32, device=DEV)
    igemm_wgrad(nhwc(g), x4, dw, 2, 3, 7, 7, stem=True)
    got = dw[:, :, :28].reshape(Co, 7, 7, 4)[..., :3].permute(0, 3, 1, 2)
    assert rel(got, wr.grad) < 5e-3
    assert dw[:, :, 28:].abs().max().item() == 0.0
    assert dw[:, :, :28].reshape(Co, 7, 7, 4)[..., 3].abs().max().item() == 0.0


@pytest.mark.parametrize("shape", [
    (32, 64, 56, 256, 1, 1, 0),    # K = 64: register-staged persistent grid, two channel panels
    (32, 256, 14, 1024, 1, 1, 0),  # K = 256: 256x256 LDS-DMA persistent grid, four panels
    (128, 256, 28, 64, 1, 1, 0),   # Nout = 64: one panel per block for its whole life
])
def test_conv_stats_persistent_blocks(shape):
    """Short-K convs run on a persistent grid (blocks walk many tiles) and carry
    their BN statistics in registers across a channel panel: the slab must
    still hold exactly the sums of the stored bf16 output."""
    from imagent_amd.ops.conv import igemm_fwd
    N, Ci, H, Co, k, s, p = shape
    torch.manual_seed(4)
    x = bf(torch.randn(N, H, H, Ci, device=DEV))
    w = bf(torch.randn(Co, k, k, Ci, device=DEV) * (2.0 / (Ci * k * k)) ** 0.5)
    slab = torch.zeros(32, 2, Co, device=DEV)
    y = igemm_fwd(x, w, s, p, k, k, stats=slab)
    ref = F.conv2d(nchw(x).float(), nchw(w).float(), None, s, p)
    assert rel(nchw(y), ref) < 1e-2
    yb = y.float().reshape(-1, Co)
    st = slab.sum(0)
    assert rel(st[0], yb.sum(0)) < 1e-4
    assert rel(st[1], (yb * yb).sum(0)) < 1e-4


def test_stem_stats_persistent_blocks():
    """Full-size stem (224^2 -> 112^2, 16 images): persistent grid, one channel panel."""
    from imagent_amd.ops.conv import igemm_fwd
    torch.manual_seed(8)
    N, H, Co = 16, 224, 64
    x4 = torch.zeros(N, H, H, 4, device=DEV, dtype=torch.bfloat16)
    x4[..., :3] = bf(torch.randn(N, H, H, 3, device=DEV))
    wrow = torch.zeros(Co, 7, 32, device=DEV, dtype=torch.bfloat16)
    w3 = bf(torch.randn(Co, 3, 7, 7, device=DEV) * 0.1)
    wrow[:, :, :28].view(Co, 7, 7, 4)[..., :3] = w3.permute(0, 2, 3, 1)
    slab = torch.zeros(32, 2, Co, device=DEV)
    y = igemm_fwd(x4, wrow, 2, 3, 7, 7, stats=slab, stem=True)
    ref = F.conv2d(nchw(x4[..., :3]).float(), w3.float(), None, 2, 3)
    assert rel(nchw(y), ref) < 1e-2
    yb = y.float().reshape(-1, Co)
    assert rel(slab.sum(0)[0], yb.sum(0)) < 1e-4
    assert rel(slab.sum(0)[1], (yb * yb).sum(0)) < 1e-4


@pytest.mark.parametrize("N", [1, 5])
def test_stem_band_matches_stream(N):
    """The band stem (conv_stream.hip stem_band_kernel: input rows staged in LDS once per 4 output rows, weights in
    registers) against the streaming row-segment stem (tile 23) and fp32: training forward with shifted
    statistics, and the eval forward's folded BatchNorm + ReLU; image borders on every side."""
    from imagent_amd.ops.conv import igemm_fwd
    torch.manual_seed(9)
    H, Co = 224, 64
    x4 = torch.zeros(N, H, H, 4, device=DEV, dtype=torch.bfloat16)
    x4[..., :3] = bf(torch.randn(N, H, H, 3, device=DEV) + 0.3)
    w3 = bf(torch.randn(Co, 3, 7, 7, device=DEV) * 0.1)
    wrow = torch.zeros(Co, 7, 32, device=DEV, dtype=torch.bfloat16)
    wrow[:, :, :28].view(Co, 7, 7, 4)[..., :3] = w3.permute(0, 2, 3, 1)
    ref = F.conv2d(nchw(x4[..., :3]).float(), w3.float(), None, 2, 3)
    from imagent_amd.models.resnet import BNWork
    from imagent_amd.ops import _lib
    shift = torch.randn(Co, device=DEV) * 0.1
    outs = {}
    for tile in (0, 23):
        work = BNWork(torch.zeros(32, 2, Co, device=DEV), torch.zeros(2, Co, device=DEV),
                      torch.stack([shift, torch.ones(Co, device=DEV)]),
                      torch.zeros(_lib.kernels().imk_bn_bwd_scratch_floats(Co), device=DEV))
        y = igemm_fwd(x4, wrow, 2, 3, 7, 7, stats=work, stem=True, tile=tile)
        outs[tile] = (y, work.slab.sum(0))
    y0, st0 = outs[0]
    y1, st1 = outs[23]
    assert rel(nchw(y0), ref) < 1e-2
    assert rel(y0.float(), y1.float()) < 1e-3
    d = y0.float().reshape(-1, Co) - shift
    assert rel(st0[0], d.sum(0)) < 1e-4 and rel(st0[1], (d * d).sum(0)) < 1e-4
    # eval: folded BN (scale, shift) + ReLU in the epilogue
    aff = torch.stack([torch.rand(Co, device=DEV) + 0.5, torch.randn(Co, device=DEV) * 0.2]).contiguous()
    ye = igemm_fwd(x4, wrow, 2, 3, 7, 7, stem=True, affine=aff, relu=True)
    want = torch.relu(y0.float() * aff[0] + aff[1])
    assert rel(ye.float(), want) < 1e-2


def test_maxpool_stem_size():
    """The stem's pool at a full-size row (112 px, 64 ch): row-grid indexing."""
    from imagent_amd.ops.misc import MaxPoolFn
    torch.manual_seed(5)
    x = bf(torch.randn(3, 112, 112, 64, device=DEV)).requires_grad_(True)
    y = MaxPoolFn.apply(x, 3, 2, 1)
    xr = nchw(x.detach()).float().requires_grad_(True)
    yr = F.max_pool2d(xr, 3, 2, 1)
    assert torch.equal(nchw(y).float(), yr)
    g = bf(torch.randn_like(y))
    y.backward(g)
    yr.backward(nchw(g).float())
    assert rel(nchw(x.grad), xr.grad) < 1e-2


def test_conv_fwd_bias_fp32_out():
    from imagent_amd.ops.conv import igemm_fwd
    torch.manual_seed(1)
    x = bf(torch.randn(16, 512, device=DEV))
    w = bf(torch.randn(1000, 512, device=DEV) * 0.05)
    b = torch.randn(1000, device=DEV)
    y = igemm_fwd(x.view(16, 1, 1, 512), w.view(1000, 1, 1, 512), 1, 0, 1, 1, bias=b, out_f32=True)
    ref = x.float() @ w.float().t() + b
    assert y.dtype == torch.float32
    assert rel(y.view(16, 1000), ref) < 1e-4


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("C", [64, 256, 2048])
def test_bn_fwd_bwd(mode, C):
    from imagent_amd.models.resnet import BatchNorm2d, BNWork
    from imagent_amd.ops import _lib
    from imagent_amd.ops.bn import BNActFn
    torch.manual_seed(2)
    N, H = 4, 7
    x = bf(torch.randn(N, H, H, C, device=DEV) * 2 + 0.5)
    x2 = bf(torch.randn(N, H, H, C, device=DEV))
    bn = BatchNorm2d(C).to(DEV)
    bn2 = BatchNorm2d(C).to(DEV)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
        bn2.weight.uniform_(0.5, 1.5)
        bn2.bias.uniform_(-0.5, 0.5)
    for m in (bn, bn2):
        m.weight.grad = torch.zeros_like(m.weight)
        m.bias.grad = torch.zeros_like(m.bias)
    for m, t in ((bn, x), (bn2, x2)):
        slab = torch.zeros(32, 2, C, device=DEV)
        slab[3] = torch.stack([t.float().sum((0, 1, 2)), (t.float() ** 2).sum((0, 1, 2))])
        nbw = _lib.kernels().imk_bn_bwd_scratch_floats(C)
        m.work = BNWork(slab, torch.zeros(2, C, device=DEV), torch.zeros(2, C, device=DEV),
                        torch.zeros(nbw, device=DEV))
    xa = x.clone().requires_grad_(True)
    x2a = x2.clone().requires_grad_(True)
    y = BNActFn.apply(xa, x2a if mode else None, bn, bn2 if mode == 2 else None, mode, True)
    g = bf(torch.randn_like(y.float()))
    y.backward(g)

    # reference
    xr = nchw(x).float().requires_grad_(True)
    x2r = nchw(x2).float().requires_grad_(True)
    gr_w = bn.weight.detach().clone().requires_grad_(True)
    gr_b = bn.bias.detach().clone().requires_grad_(True)
    gr_w2 = bn2.weight.detach().clone().requires_grad_(True)
    gr_b2 = bn2.bias.detach().clone().requires_grad_(True)
    yr = F.batch_norm(xr, None, None, gr_w, gr_b, True, 0.1, 1e-5)
    if mode == 1:
        yr = yr + x2r
    elif mode == 2:
        yr = yr + F.batch_norm(x2r, None, None, gr_w2, gr_b2, True, 0.1, 1e-5)
    yr = F.relu(yr)
    yr.backward(nchw(g).float())
    assert rel(nchw(y), yr) < 1e-2
    assert rel(nchw(xa.grad), xr.grad) < 2e-2
    assert rel(bn.weight.grad, gr_w.grad) < 1e-2
    assert rel(bn.bias.grad, gr_b.grad) < 1e-2
    if mode == 1:
        assert rel(nchw(x2a.grad), x2r.grad) < 1e-2
    if mode == 2:
        assert rel(nchw(x2a.grad), x2r.grad) < 2e-2
        assert rel(bn2.weight.grad, gr_w2.grad) < 1e-2
        assert rel(bn2.bias.grad, gr_b2.grad) < 1e-2


def test_maxpool_avgpool():
    from imagent_amd.ops.misc import AvgPoolFn, MaxPoolFn
    torch.manual_seed(3)
    x = bf(torch.randn(2, 64, 17, 17, device=DEV))
    xa = nhwc(x).requires_grad_(True)
    y = MaxPoolFn.apply(xa, 3, 2, 1)
    g = bf(torch.randn_like(y.float()))
    y.backward(g)
    xr = x.float().requires_grad_(True)
    yr = F.max_pool2d(xr, 3, 2, 1)
    yr.backward(nchw(g).float())
    assert rel(nchw(y), yr) == 0.0
    assert rel(nchw(xa.grad), xr.grad) < 1e-2

    x = bf(torch.randn(3, 7, 7, 256, device=DEV)).requires_grad_(True)
    p = AvgPoolFn.apply(x)
    assert rel(p, x.float().mean((1, 2))) < 1e-2
    gp = bf(torch.randn(3, 256, device=DEV))
    p.backward(gp)
    assert rel(x.grad, gp.float()[:, None, None, :].expand(3, 7, 7, 256) / 49) < 1e-2


def test_xent_topk():
    from imagent_amd.ops.misc import XentFn
    torch.manual_seed(4)
    z = torch.randn(64, 1000, device=DEV) * 3
    lab = torch.randint(0, 1000, (64,), device=DEV)
    lab[:8] = z[:8].argmax(1)  # force some top-1 hits
    met = torch.zeros(4, device=DEV)
    za = z.clone().requires_grad_(True)
    loss = XentFn.apply(za, lab, met, 0.0)
    loss.backward()
    zr = z.clone().requires_grad_(True)
    lr = F.cross_entropy(zr, lab)
    lr.backward()
    assert abs(loss.item() - lr.item()) < 1e-4
    assert rel(za.grad, zr.grad) < 1e-2
    top5 = z.topk(5, 1).indices
    assert met[1].item() == (top5[:, 0] == lab).sum().item()
    assert met[2].item() == (top5 == lab[:, None]).any(1).sum().item()
    assert met[3].item() == 64
    assert abs(met[0].item() - lr.item() * 64) < 1e-2


def test_sgd_flat_matches_torch():
    from imagent_amd.ops.misc import sgd_flat
    torch.manual_seed(5)
    n = 10007
    p = torch.randn(n, device=DEV)
    ps = [p.clone().requires_grad_(True)]
    opt = torch.optim.SGD(ps, lr=0.1, momentum=0.9, weight_decay=1e-4)
    buf = torch.zeros(n, device=DEV)
    sh = torch.empty(n, device=DEV, dtype=torch.bfloat16)
    for step in range(3):
        g = torch.randn(n, device=DEV)
        ps[0].grad = g.clone()
        opt.step()
        sgd_flat(p, g, buf, sh, 0.1, 0.9, 0.0, 1e-4, False, step == 0)
    assert rel(p, ps[0].detach()) < 1e-6
    assert rel(sh, p) < 1e-2


def test_normalize_and_transpose():
    from imagent_amd.ops.misc import TransposePlan, normalize_u8
    torch.manual_seed(6)
    img = torch.randint(0, 256, (3, 40, 50, 3), dtype=torch.uint8, device=DEV)
    crop = torch.tensor([[1, 2], [0, 0], [5, 7]], dtype=torch.int32, device=DEV)
    flip = torch.tensor([0, 1, 1], dtype=torch.uint8, device=DEV)
    out = normalize_u8(img, (32, 40), 8, (0.5, 0.5, 0.5), (0.5, 0.5, 0.5), crop, flip)
    ref = torch.zeros(3, 32, 40, 8, device=DEV)
    for b in range(3):
        oy, ox = crop[b].tolist()
        t = img[b, oy:oy + 32, ox:ox + 40].float() / 255
        if flip[b]:
            t = t.flip(1)
        ref[b, ..., :3] = (t - 0.5) / 0.5
    assert rel(out, ref) < 5e-3
    a = bf(torch.randn(96, 9, 40, device=DEV))
    b = torch.empty(40, 9, 96, device=DEV, dtype=torch.bfloat16)
    c = bf(torch.randn(1000, 1, 64, device=DEV))
    d = torch.empty(64, 1, 1000, device=DEV, dtype=torch.bfloat16)
    TransposePlan([(a, b, 96, 9, 40), (c, d, 1000, 1, 64)], DEV).run()
    assert torch.equal(b, a.permute(2, 1, 0))
    assert torch.equal(d, c.permute(2, 1, 0))


@pytest.mark.parametrize("W,Cp", [(40, 4), (36, 8), (38, 4), (38, 8)])
def test_normalize_quad_and_per_pixel_paths(W, Cp):
    """The 4-pixel normalize kernel (W % 4 == 0, Cp 4 / 8) and the per-pixel one (W = 38) against torch, with
    per-sample crops and flips."""
    from imagent_amd.ops.misc import normalize_u8
    torch.manual_seed(7)
    img = torch.randint(0, 256, (4, 41, 47, 3), dtype=torch.uint8, device=DEV)
    crop = torch.tensor([[1, 2], [0, 0], [5, 7], [9, 47 - W]], dtype=torch.int32, device=DEV)
    flip = torch.tensor([0, 1, 1, 0], dtype=torch.uint8, device=DEV)
    mean, std = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)
    out = normalize_u8(img, (32, W), Cp, mean, std, crop, flip).float()
    ref = torch.zeros(4, 32, W, Cp, device=DEV)
    for b in range(4):
        oy, ox = crop[b].tolist()
        t = img[b, oy:oy + 32, ox:ox + W].float() / 255
        if flip[b]:
            t = t.flip(1)
        ref[b, ..., :3] = (t - torch.tensor(mean, device=DEV)) / torch.tensor(std, device=DEV)
    assert (out - ref).abs().max().item() < 0.02  # bf16 rounding of values up to |2.6|
    assert torch.equal(out[..., 3:], torch.zeros_like(out[..., 3:]))


def test_fp8_quant_matches_torch_e4m3():
    from imagent_amd.ops.fp8 import ActScales, WeightQuantizer, quant_act
    torch.manual_seed(8)
    x = bf(torch.randn(4096, device=DEV) * 3)
    sc = ActScales(1, DEV)
    sc.exp.fill_(-2)  # q = x * 4
    q = quant_act(x, sc.exp[0:1], sc.amax[0])
    ref = (x.float() * 4).clamp(-448, 448).to(torch.float8_e4m3fn)
    assert torch.equal(q, ref.view(torch.uint8))
    assert sc.amax.max().item() == x.float().abs().max().item()
    sc.step()  # amax ~ 12 -> exponent ceil(log2(12/448)) = -5
    assert sc.exp.item() == -5 and sc.amax.abs().max().item() == 0.0
    w = torch.randn(64, 32, 3, 3, device=DEV).contiguous(memory_format=torch.channels_last)
    wq = WeightQuantizer([w], DEV)
    wq.run()
    e = wq.exp.item()
    amax = w.abs().max().item()
    assert amax * 2.0 ** -e <= 448 and amax * 2.0 ** -(e - 1) > 448
    w_nhwc = w.permute(0, 2, 3, 1).contiguous().flatten()
    ref = (w_nhwc * 2.0 ** -e).to(torch.float8_e4m3fn).view(torch.uint8)
    assert torch.equal(wq.views[0], ref)


@pytest.mark.parametrize("epi", [0, 1, 2])
@pytest.mark.parametrize("tile", [0, 2, 4, 8, 17, 18, 19])
@pytest.mark.parametrize("shape", [(4, 64, 14, 128, 3, 1, 1), (2, 256, 9, 512, 1, 2, 0), (3, 16, 11, 64, 3, 1, 1),
                                   (2, 128, 14, 256, 1, 1, 0), (4, 64, 16, 64, 3, 1, 1), (2, 512, 4, 512, 3, 1, 1)])
def test_conv_fp8_forward(tile, shape, epi):
    """Block-scaled fp8 MFMA conv vs fp32 conv of the same dequantised operands (tiles 17 / 18 / 19: the
    v3 main loop with 1-byte operands, C % 128 == 0 and the staged epilogue only; tile 0 takes it there)."""
    from imagent_amd.ops.conv import igemm_fwd
    N, Ci, H, Co, k, s, p = shape
    if tile >= 17 and (Ci % 128 or epi == 1):
        pytest.skip("v3 fp8: C % 128 == 0, staged epilogue")
    torch.manual_seed(9)
    ex, ew = -3, -8
    x = torch.randn(N, H, H, Ci, device=DEV).abs() * 4  # post-ReLU-like
    w = torch.randn(Co, k, k, Ci, device=DEV) * 0.05
    x8 = (x * 2.0 ** -ex).clamp(-448, 448).to(torch.float8_e4m3fn)
    w8 = (w * 2.0 ** -ew).clamp(-448, 448).to(torch.float8_e4m3fn)
    xd = x8.float() * 2.0 ** ex
    wd = w8.float() * 2.0 ** ew
    yr = F.conv2d(nchw(xd), wd.permute(0, 3, 1, 2), None, s, p)
    slab = torch.zeros(32, 2, Co, device=DEV)
    e = torch.tensor([ex, ew], dtype=torch.int32, device=DEV)
    y = igemm_fwd(x8.view(torch.uint8), w8.view(torch.uint8), s, p, k, k, stats=slab, tile=tile,
                  fp8=(e[0:1], e[1:2]), epi=epi)
    assert rel(nchw(y), yr) < 1e-2
    yb = nchw(y).float()
    assert rel(slab.sum(0)[0], yb.sum((0, 2, 3))) < 1e-3


def test_lars_native_matches_cpu_math():
    import torch.nn as nn

    from imagent_amd.models.arena import ParamArena
    from imagent_amd.train.optim import FlatLARS
    torch.manual_seed(3)
    nets = [nn.Sequential(nn.Conv2d(16, 32, 3), nn.BatchNorm2d(32), nn.Flatten(), nn.Linear(32, 10))
            for _ in range(2)]
    nets[1].load_state_dict(nets[0].state_dict())
    ar_g = ParamArena(list(nets[0].named_parameters()), torch.device(DEV), with_shadow=True)
    ar_c = ParamArena(list(nets[1].named_parameters()), torch.device("cpu"))
    og = FlatLARS(ar_g, lr=2.0, momentum=0.9, weight_decay=5e-5, eta=1e-3)
    oc = FlatLARS(ar_c, lr=2.0, momentum=0.9, weight_decay=5e-5, eta=1e-3, native=False)
    assert og.native
    for _ in range(3):
        g = torch.randn(ar_c.total)
        ar_c.G.copy_(g)
        ar_g.G.copy_(g.to(DEV))
        og.step()
        oc.step()
    assert torch.allclose(ar_g.P.cpu(), ar_c.P, rtol=1e-4, atol=1e-6)
    assert torch.equal(ar_g.S.cpu(), ar_g.P.cpu().to(torch.bfloat16))


@pytest.mark.parametrize("accum", [False, True])
@pytest.mark.parametrize("shape", [(4, 64, 14, 128, 3, 1, 1), (2, 256, 9, 512, 1, 2, 0), (3, 128, 12, 64, 3, 2, 1),
                                   (2, 512, 7, 256, 1, 1, 0)])
def test_conv_fp8_dgrad(shape, accum):
    """e5m2 gradient x e4m3 transposed weights (IG_FP8 | IG_BF8X) vs the fp32
    dgrad of the dequantised operands, incl. strided parity classes and the
    residual-accumulating epilogue."""
    from imagent_amd.ops.conv import igemm_dgrad
    N, Ci, H, Co, k, s, p = shape
    torch.manual_seed(13)
    eg, ew = -14, -9
    w = torch.randn(Co, Ci, k, k, device=DEV) * 0.05
    OH = (H + 2 * p - k) // s + 1
    g = torch.randn(N, Co, OH, OH, device=DEV) * 1e-3
    g8 = (g * 2.0 ** -eg).clamp(-57344, 57344).to(torch.float8_e5m2)
    w8 = (w * 2.0 ** -ew).clamp(-448, 448).to(torch.float8_e4m3fn)
    gd, wd = g8.float() * 2.0 ** eg, w8.float() * 2.0 ** ew
    xr = torch.zeros(N, Ci, H, H, device=DEV, requires_grad=True)
    F.conv2d(xr, wd, None, s, p).backward(gd)
    e = torch.tensor([eg, ew], dtype=torch.int32, device=DEV)
    wt8 = w8.view(torch.uint8).permute(1, 2, 3, 0).contiguous()  # [Ci][KH][KW][Co]
    dy_bf = nhwc(bf(gd))  # the bf16 operand only provides shapes here
    base = bf(torch.randn(N, H, H, Ci, device=DEV) * 1e-3) if accum else None
    out = base.clone() if accum else None
    dx = igemm_dgrad(dy_bf, wt8, (H, H), s, p, k, k, out=out, accumulate=accum,
                     fp8=(nhwc(g8.view(torch.uint8)), e[0:1], wt8, e[1:2]))
    ref = nhwc(xr.grad) + (base.float() if accum else 0)
    assert rel(dx, ref) < 1e-2


@pytest.mark.parametrize("H", [30, 31, 56])
def test_maxpool_bwd_bn_reduce_fused(H):
    """imk_maxpool_bwd_bnr: pool backward + ReLU mask from x + BN-backward sums
    (even H: the 2x2-quad kernel of the stem pool; odd H: the per-pixel one)."""
    from imagent_amd.ops import _lib
    from imagent_amd.ops.misc import MaxPoolFn
    torch.manual_seed(7)
    N, C = 4, 64
    x = bf(torch.randn(N, H, H, C, device=DEV))
    mean, rstd = torch.randn(C, device=DEV) * 0.1, torch.rand(C, device=DEV) + 0.5
    gamma, beta = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV) * 0.2
    h = torch.relu((x.float() - mean) * rstd * gamma + beta).to(torch.bfloat16).requires_grad_(True)
    y = MaxPoolFn.apply(h, 3, 2, 1)
    dy = bf(torch.randn_like(y.float()))
    y.backward(dy)
    g_ref = h.grad.float() * ((x.float() - mean) * rstd * gamma + beta > 0)
    OH = y.shape[1]
    idx = torch.empty(y.shape, dtype=torch.uint8, device=DEV)
    tmp = torch.empty_like(y)
    _lib.check(_lib.kernels().imk_maxpool_fwd(h.detach().data_ptr(), tmp.data_ptr(), idx.data_ptr(), N, H, H, C,
                                              OH, OH, 3, 2, 1, _lib.stream_ptr()), "pool")
    save = torch.stack([mean, rstd]).contiguous()
    slab = torch.zeros(32, 3, C, device=DEV)
    g = torch.empty_like(x)
    _lib.check(_lib.kernels().imk_maxpool_bwd_bnr(dy.data_ptr(), idx.data_ptr(), g.data_ptr(), x.data_ptr(),
                                                  None, save.data_ptr(), gamma.data_ptr(), beta.data_ptr(),
                                                  slab.data_ptr(), N, H, H, C, OH, OH, 3, 2, 1,
                                                  _lib.stream_ptr()), "pool bwd bnr")
    assert rel(g, g_ref) < 1e-2
    gb = g.float()
    xhat = (x.float() - mean) * rstd
    s = slab.sum(0)
    assert rel(s[0], (gb * xhat).sum((0, 1, 2))) < 1e-3
    assert rel(s[1], gb.sum((0, 1, 2))) < 1e-3


@pytest.mark.parametrize("H", [30, 56])
def test_maxpool_bnr_from_argmax_input(H):
    """The stem pool's BN backward without re-reading x (StemFn): imk_maxpool_fwd_bn also stores the BN input at
    each window's argmax (xsel); imk_maxpool_bwd_bnr given xsel takes every window's ReLU mask from it and sums
    from the argmax input of a window that took each pixel -- the same gradient bit for bit as the x-reading pass,
    and the same BN sums term for term."""
    from imagent_amd.ops import _lib
    from imagent_amd.ops.misc import MaxPoolFn
    kern = _lib.kernels()
    torch.manual_seed(8)
    N, C, eps = 4, 64, 1e-5
    x = bf(torch.randn(N, H, H, C, device=DEV))
    mean, var = torch.randn(C, device=DEV) * 0.1, torch.rand(C, device=DEV) + 0.5
    gamma, beta = torch.randn(C, device=DEV), torch.randn(C, device=DEV) * 0.3  # some gamma < 0
    sums = torch.stack([mean, var]).contiguous()
    OH = (H + 2 - 3) // 2 + 1
    y = torch.empty(N, OH, OH, C, device=DEV, dtype=torch.bfloat16)
    idx = torch.empty(y.shape, dtype=torch.uint8, device=DEV)
    xsel = torch.empty_like(y)
    save = torch.empty(2, C, device=DEV)
    _lib.check(kern.imk_maxpool_fwd_bn(x.data_ptr(), sums.data_ptr(), gamma.data_ptr(), beta.data_ptr(),
                                       save.data_ptr(), y.data_ptr(), idx.data_ptr(), xsel.data_ptr(), N, H, H, C,
                                       OH, OH, 3, 2, 1, eps, _lib.stream_ptr()), "bn + pool")
    sc = save[1] * gamma
    sh = beta - save[0] * sc
    h = torch.relu(x.float() * sc + sh).to(torch.bfloat16).requires_grad_(True)
    yr = MaxPoolFn.apply(h, 3, 2, 1)
    assert rel(y, yr) < 1e-3
    # xsel holds an input of the window that maps to the pooled value
    assert rel(torch.relu(xsel.float() * sc + sh), y.float()) < 1e-2
    dy = bf(torch.randn_like(y.float()))
    gs = []
    for use_xsel in (False, True):
        slab = torch.zeros(32, 3, C, device=DEV)
        g = torch.empty_like(x)
        _lib.check(kern.imk_maxpool_bwd_bnr(dy.data_ptr(), idx.data_ptr(), g.data_ptr(), x.data_ptr(),
                                            xsel.data_ptr() if use_xsel else None, save.data_ptr(),
                                            gamma.data_ptr(), beta.data_ptr(), slab.data_ptr(), N, H, H, C, OH, OH,
                                            3, 2, 1, _lib.stream_ptr()), "pool bwd bnr")
        gs.append((g, slab.sum(0)))
    (g1, s1), (g2, s2) = gs
    assert torch.equal(g1, g2)
    yr.backward(dy)
    g_ref = h.grad.float() * (x.float() * sc + sh > 0)
    assert rel(g2, g_ref) < 1e-2
    gb = g2.float()
    xhat = (x.float() - save[0]) * save[1]
    assert rel(s2[0], (gb * xhat).sum((0, 1, 2))) < 1e-3
    assert rel(s2[1], gb.sum((0, 1, 2))) < 1e-3
    assert rel(s2[:2], s1[:2]) < 1e-5


@pytest.mark.parametrize("R,Cc", [(512, 1000), (7, 10), (100, 64), (2048, 130)])
def test_colsum_accumulates(R, Cc):
    """fc bias gradient: out += column sums of a bf16 [R, C] matrix."""
    from imagent_amd.ops.conv import colsum_into
    torch.manual_seed(9)
    x = bf(torch.randn(R, Cc, device=DEV))
    out = torch.randn(Cc, device=DEV)
    ref = out + x.float().sum(0)
    colsum_into(x, out)
    assert rel(out, ref) < 1e-5


@pytest.mark.parametrize("cmid,cin,tile,epi", [(64, 256, 0, 0), (128, 256, 0, 0), (256, 512, 0, 0),
                                               (128, 512, 8, 2), (96, 256, 2, 1), (64, 128, 4, 0)])
def test_sparse_downsample_dgrad_then_accumulate(cmid, cin, tile, epi):
    """Bottleneck downsample backward without the memset: the stride-2 1x1 dgrad writes only
    the even pixels (sparse) and conv1's dgrad accumulates treating the odd ones as zero
    (IG_ACCUM_SUB2) -- bit-identical to memset + dense accumulate, on every epilogue path."""
    from imagent_amd.ops.conv import igemm_dgrad
    torch.manual_seed(9)
    N, H = 3, 14
    cds = 2 * cin
    g_ds = bf(torch.randn(N, H // 2, H // 2, cds, device=DEV))
    w_ds = bf(torch.randn(cin, 1, 1, cds, device=DEV) * 0.05)   # [Ci][KH][KW][Co] (transposed)
    g1 = bf(torch.randn(N, H, H, cmid, device=DEV))
    w1 = bf(torch.randn(cin, 1, 1, cmid, device=DEV) * 0.1)
    ref = igemm_dgrad(g_ds, w_ds, (H, H), 2, 0, 1, 1)                     # memset + class (0, 0)
    igemm_dgrad(g1, w1, (H, H), 1, 0, 1, 1, out=ref, accumulate=True, tile=tile, epi=epi)
    got = torch.full_like(ref, float("nan"))                              # garbage where not written
    igemm_dgrad(g_ds, w_ds, (H, H), 2, 0, 1, 1, out=got, sparse=True)
    assert torch.isnan(got[:, 1::2].float()).all() and torch.isnan(got[:, :, 1::2].float()).all()
    igemm_dgrad(g1, w1, (H, H), 1, 0, 1, 1, out=got, accumulate=True, tile=tile, epi=epi, old_sub2=True)
    assert torch.equal(got, ref)


@pytest.mark.parametrize("shape", [(3, 64, 56), (2, 64, 112)])
def test_halo_conv3x3(shape):
    """64 -> 64 3x3 stride-1 convs run on the halo-tiled kernel (conv_halo.hip):
    forward with BN statistics, dgrad, accumulating dgrad vs fp32, and the
    kernel that ran is the halo kernel."""
    from torch.profiler import ProfilerActivity, profile
    from imagent_amd.ops.conv import igemm_dgrad, igemm_fwd
    N, C, H = shape
    torch.manual_seed(3)
    x = bf(torch.randn(N, C, H, H, device=DEV) + 0.5)
    w = bf(torch.randn(C, C, 3, 3, device=DEV) * (2.0 / (C * 9)) ** 0.5)
    xr = x.float().requires_grad_(True)
    yr = F.conv2d(xr, w.float(), None, 1, 1)
    g = bf(torch.randn_like(yr))
    yr.backward(g.float())
    slab = torch.zeros(32, 2, C, device=DEV)
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        y = igemm_fwd(nhwc(x), nhwc(w), 1, 1, 3, 3, stats=slab)
        wt = w.permute(1, 2, 3, 0).contiguous()
        dx = igemm_dgrad(nhwc(g), wt, (H, H), 1, 1, 3, 3)
        torch.cuda.synchronize()
    names = [e.name for e in prof.events() if "halo3x3_kernel" in e.name]
    assert len(names) >= 2, [e.name for e in prof.events() if "kernel" in e.name][:8]
    assert rel(nchw(y), yr) < 1e-2
    yb = nchw(y).float()
    st = slab.sum(0)
    assert rel(st[0], yb.sum((0, 2, 3))) < 1e-3 and rel(st[1], (yb * yb).sum((0, 2, 3))) < 1e-3
    assert rel(nchw(dx), xr.grad) < 1e-2
    # accumulate: dx += dgrad again
    base = dx.clone()
    igemm_dgrad(nhwc(g), wt, (H, H), 1, 1, 3, 3, out=dx, accumulate=True)
    assert rel(dx.float() - base.float(), nhwc(xr.grad)) < 2e-2




@pytest.mark.parametrize("variant", ["y_mask", "x_mask", "x2"])
@pytest.mark.parametrize("N,H", [(3, 56), (2, 112)])
def test_halo_dgrad_bnb_matches_tiled(N, H, variant):
    """The halo kernel's fused BatchNorm-backward dgrad epilogue (EPI 1: x / mask-bit operands prefetched before the
    next band's patch at W = 56; EPI 2: the second BN branch) against the tiled kernel (tile 1) on the same
    operands: stored gradient and the three slab reductions."""
    from imagent_amd.models.resnet import BatchNorm2d, BNWork
    from imagent_amd.ops import _lib
    from imagent_amd.ops.bn import relu_mask_bits
    from imagent_amd.ops.conv import BNBwdFuse, igemm_dgrad
    from torch.profiler import ProfilerActivity, profile
    C = 64
    torch.manual_seed(11)
    dy = bf(torch.randn(N, H, H, C, device=DEV))
    wt = bf(torch.randn(C, 3, 3, C, device=DEV) * (1.0 / (9 * C)) ** 0.5)
    x = bf(torch.randn(N, H, H, C, device=DEV))
    y = bf(torch.randn(N, H, H, C, device=DEV)) if variant in ("y_mask", "x2") else None
    x2 = bf(torch.randn(N, H, H, C, device=DEV)) if variant == "x2" else None
    nbw = _lib.kernels().imk_bn_bwd_scratch_floats(1)

    def mk():
        bn = BatchNorm2d(C).to(DEV)
        with torch.no_grad():
            bn.weight.uniform_(0.5, 1.5)
            bn.bias.uniform_(-0.2, 0.2)
        save = torch.stack([torch.randn(C, device=DEV) * 0.1, torch.rand(C, device=DEV) + 0.5])
        bn.work = BNWork(None, None, save, torch.zeros(nbw * C, device=DEV))
        return bn

    bn, bn2 = mk(), mk()
    outs = []
    for tile in (0, 1):
        bn.work.scratch.zero_()
        f = BNBwdFuse(x, bn, y=relu_mask_bits(y) if y is not None else None, x2=x2, bn2=bn2 if x2 is not None else None)
        with profile(activities=[ProfilerActivity.CUDA]) as prof:
            r = igemm_dgrad(dy, wt, (H, H), 1, 1, 3, 3, bnb=f, tile=tile)
            torch.cuda.synchronize()
        halo = any("halo3x3_kernel" in e.name for e in prof.events())
        assert halo == (tile == 0), tile
        outs.append((r.clone(), bn.work.scratch[:32 * 3 * C].view(32, 3, C).sum(0).clone()))
    (r0, s0), (r1, s1) = outs
    assert rel(r0, r1) < 5e-3
    for q in range(3 if x2 is not None else 2):
        assert rel(s0[q], s1[q]) < 2e-3, q
