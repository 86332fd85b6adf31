"""Streaming short-K 1x1 conv kernel (csrc/kernels/conv_stream.hip) vs the
fp32 PyTorch reference and vs the tiled implicit-GEMM kernels it replaces
for those shapes (forward + BN statistics, IG_ACCUM, dgrad with the fused
BN-backward epilogue)."""

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


def nchw(t):
    return t.permute(0, 3, 1, 2).contiguous()


@pytest.fixture
def stream_toggle():
    from imagent_amd.ops import conv
    yield conv.set_stream
    conv.set_stream(True)


SHAPES = [
    # N, Ci, H, Co, stride
    (8, 64, 56, 256, 1),
    (5, 64, 13, 64, 1),     # ragged pixel count (M % 16 != 0)
    (6, 64, 15, 192, 1),    # Nout not a multiple of 128 -> 64-channel slices
    (4, 128, 28, 512, 1),
    (3, 128, 11, 128, 1),
    (4, 64, 28, 128, 2),    # strided 1x1 (ResNet-18/34 downsample): pixel gather
    (6, 256, 14, 64, 1),    # K = 256 into 64 channels
    (3, 256, 13, 128, 1),   # K = 256, two 64-channel slices, ragged pixels
]


@pytest.mark.parametrize("tile", [0, 21, 22])
@pytest.mark.parametrize("shape", SHAPES)
def test_stream_fwd_stats(shape, tile):
    from imagent_amd.ops.conv import igemm_fwd
    N, Ci, H, Co, s = shape
    torch.manual_seed(1)
    x = torch.randn(N, H, H, Ci, device=DEV).to(torch.bfloat16)
    w = (torch.randn(Co, 1, 1, Ci, device=DEV) * (2.0 / Ci) ** 0.5).to(torch.bfloat16)
    slab = torch.zeros(32, 2, Co, device=DEV)
    y = igemm_fwd(x, w, s, 0, 1, 1, stats=slab, tile=tile)
    ref = F.conv2d(nchw(x).float(), nchw(w).float(), None, s, 0)
    assert rel(nchw(y), ref) < 1e-2
    yb = y.float().reshape(-1, Co)
    st = slab.sum(0)
    assert rel(st[0], yb.sum(0)) < 1e-4
    assert rel(st[1], (yb * yb).sum(0)) < 1e-4


def test_stream_fwd_accumulate():
    from imagent_amd.ops.conv import igemm_fwd
    torch.manual_seed(2)
    x = torch.randn(4, 20, 20, 64, device=DEV).to(torch.bfloat16)
    w = (torch.randn(256, 1, 1, 64, device=DEV) * 0.1).to(torch.bfloat16)
    base = torch.randn(4, 20, 20, 256, device=DEV).to(torch.bfloat16)
    out = base.clone()
    igemm_fwd(x, w, 1, 0, 1, 1, out=out, accumulate=True)
    ref = nchw(base).float() + F.conv2d(nchw(x).float(), nchw(w).float())
    assert rel(nchw(out), ref) < 1e-2


@pytest.mark.parametrize("variant", ["y_mask", "x_mask", "x2", "accum"])
@pytest.mark.parametrize("shape", [(8, 64, 28, 256), (3, 128, 9, 512), (5, 64, 13, 64), (4, 256, 14, 64),
                                   (3, 256, 9, 128)])
def test_stream_dgrad_bnb_matches_tiled(shape, variant, stream_toggle):
    """dX = dY x W^T for a 1x1 conv with K = Cout in {64, 128}, through the
    IG_BNBWD epilogue: stored gradient and slab reductions must match the
    tiled kernel's (itself tested against PyTorch in test_model_gpu)."""
    from imagent_amd.models.resnet import BatchNorm2d, BNWork
    from imagent_amd.ops import _lib
    from imagent_amd.ops.bn import relu_mask_bits
    from imagent_amd.ops.conv import BNBwdFuse, igemm_dgrad
    N, Co, H, Ci = shape  # conv Ci -> Co; the dgrad output has Ci channels
    torch.manual_seed(3)
    dy = torch.randn(N, H, H, Co, device=DEV).to(torch.bfloat16)
    wt = (torch.randn(Ci, 1, 1, Co, device=DEV) * (1.0 / Co) ** 0.5).to(torch.bfloat16)
    x = torch.randn(N, H, H, Ci, device=DEV).to(torch.bfloat16)
    y = torch.randn(N, H, H, Ci, device=DEV).to(torch.bfloat16) if variant in ("y_mask", "x2", "accum") else None
    x2 = torch.randn(N, H, H, Ci, device=DEV).to(torch.bfloat16) if variant == "x2" else None
    old = torch.randn(N, H, H, Ci, device=DEV).to(torch.bfloat16) if variant == "accum" else None
    nbw = _lib.kernels().imk_bn_bwd_scratch_floats(1)

    def mk():
        bn = BatchNorm2d(Ci).to(DEV)
        with torch.no_grad():
            bn.weight.uniform_(0.5, 1.5)
            bn.bias.uniform_(-0.2, 0.2)
        save = torch.stack([torch.randn(Ci, device=DEV) * 0.1, torch.rand(Ci, device=DEV) + 0.5])
        bn.work = BNWork(None, None, save, torch.zeros(nbw * Ci, device=DEV))
        return bn

    bn, bn2 = mk(), mk()
    outs = []
    for stream in (False, True):
        stream_toggle(stream)
        bn.work.scratch.zero_()
        out = old.clone() if old is not None else None
        f = BNBwdFuse(x, bn, y=relu_mask_bits(y) if y is not None else None, x2=x2, bn2=bn2 if x2 is not None else None)
        r = igemm_dgrad(dy, wt, (H, H), 1, 0, 1, 1, out=out, accumulate=old is not None, bnb=f)
        outs.append((r.clone(), bn.work.scratch[:32 * 3 * Ci].view(32, 3, Ci).sum(0).clone()))
    (r0, s0), (r1, s1) = outs
    assert rel(r1, r0) < 5e-3
    for q in range(3 if x2 is not None else 2):
        assert rel(s1[q], s0[q]) < 2e-3, q
    # and the raw product against fp32 PyTorch (masked entries are zero in both)
    g = torch.einsum("nhwk,ck->nhwc", dy.float(), wt.view(Ci, Co).float())
    if old is not None:
        g = g + old.float()
    keep = r1.float() != 0
    assert rel(r1.float()[keep], g[keep]) < 1e-2
