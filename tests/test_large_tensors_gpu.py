"""Kernels on tensors past 2^31 bytes (a batch of 2048 images at 224 px puts 3.3 GB in one layer-1 activation).

The GEMM-shaped kernels address their operands through 32-bit buffer offsets from a descriptor base; that base
is per tile (v3 conv), per split (weight gradients), per band (halo kernels) or per pixel group (streaming 1x1),
so any tensor size works. Each test runs a kernel on cat([x, x]) (> 2 GB) and checks the two halves against each
other and against the same kernel on x alone: per-pixel results (forward, dgrad) bit for bit, the weight gradient
as 2 x the half's up to summation order. (A whole-network comparison cannot do this: a random-init ResNet-50's
gradient differs by O(1) between two runs of the SAME step, through the float-atomic summation order.)"""

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"
GB2 = 2 ** 31


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


def _pair(n, h, c, seed):
    torch.manual_seed(seed)
    x = torch.randn(n, h, h, c, device=DEV).to(torch.bfloat16)
    x2 = torch.cat([x, x])
    assert x2.numel() * 2 > GB2
    return x, x2


def _halves_equal(y2, y):
    n = y.shape[0]
    assert torch.equal(y2[:n], y2[n:]), "the two halves differ"
    assert torch.equal(y2[:n], y), "the large launch differs from the small one"


@pytest.mark.parametrize("tile", [17, 18])
def test_v3_conv_past_2gb(tile):
    """v3 main loop (explicit tiles: 256x256 / 128x128), 3x3 256 -> 256 @14 forward and dgrad."""
    from imagent_amd.ops.conv import igemm_dgrad, igemm_fwd
    x, x2 = _pair(22000, 14, 256, 1)
    w = (torch.randn(256, 3, 3, 256, device=DEV) * 0.02).to(torch.bfloat16)
    _halves_equal(igemm_fwd(x2, w, 1, 1, 3, 3, tile=tile), igemm_fwd(x, w, 1, 1, 3, 3, tile=tile))
    wt = w.permute(3, 1, 2, 0).contiguous()  # [Ci][KH][KW][Co]
    _halves_equal(igemm_dgrad(x2, wt, (14, 14), 1, 1, 3, 3, tile=tile), igemm_dgrad(x, wt, (14, 14), 1, 1, 3, 3, tile=tile))


def test_stream_conv_past_2gb():
    """streaming 1x1 kernel (K = 256 -> 64 and 64 -> 256 @56, batch 2 x 1100)."""
    from imagent_amd.ops.conv import igemm_fwd
    x, x2 = _pair(1100, 56, 256, 2)
    w = (torch.randn(64, 1, 1, 256, device=DEV) * 0.05).to(torch.bfloat16)
    _halves_equal(igemm_fwd(x2, w, 1, 0, 1, 1), igemm_fwd(x, w, 1, 0, 1, 1))
    h, h2 = x[..., :64].contiguous(), x2[..., :64].contiguous()
    w3 = (torch.randn(256, 1, 1, 64, device=DEV) * 0.1).to(torch.bfloat16)
    _halves_equal(igemm_fwd(h2, w3, 1, 0, 1, 1), igemm_fwd(h, w3, 1, 0, 1, 1))


def test_halo_conv_past_2gb():
    """halo-tiled 64 -> 64 3x3 @56 forward and dgrad."""
    from imagent_amd.ops.conv import igemm_dgrad, igemm_fwd
    x, x2 = _pair(5600, 56, 64, 3)
    w = (torch.randn(64, 3, 3, 64, device=DEV) * 0.05).to(torch.bfloat16)
    _halves_equal(igemm_fwd(x2, w, 1, 1, 3, 3), igemm_fwd(x, w, 1, 1, 3, 3))
    wt = w.permute(3, 1, 2, 0).contiguous()
    _halves_equal(igemm_dgrad(x2, wt, (56, 56), 1, 1, 3, 3), igemm_dgrad(x, wt, (56, 56), 1, 1, 3, 3))


@pytest.mark.parametrize("variant,shape", [(1, (22000, 14, 256, 256, 1)), (0, (5600, 56, 64, 64, 3)),
                                           (-1, (1100, 56, 256, 64, 1))],
                         ids=["wgrad_v3_1x1", "wgrad_halo_3x3", "wgrad_regstaged_1x1"])
def test_wgrad_past_2gb(variant, shape):
    """weight gradients (LDS-DMA v3 / halo-tiled / register-staged) over > 2 GB operands: dW(cat) = 2 dW(half)."""
    from imagent_amd.ops.conv import igemm_wgrad
    n, h, ci, co, k = shape
    x, x2 = _pair(n, h, ci, 4)
    torch.manual_seed(5)
    g = torch.randn(n, h, h, co, device=DEV).to(torch.bfloat16)
    g2 = torch.cat([g, g])
    dw = torch.zeros(co, k * k * ci, device=DEV)
    dw2 = torch.zeros_like(dw)
    igemm_wgrad(g, x, dw, 1, k // 2, k, k, variant=variant)
    igemm_wgrad(g2, x2, dw2, 1, k // 2, k, k, variant=variant)
    assert rel(dw2, 2 * dw) < 1e-3


def test_r50_forward_4096_duplicated():
    """A 4096-image ResNet-50 forward (no grad: the eval path with folded BatchNorm; layer-1 activations and the
    stem output past 2^31 ELEMENTS, 3.3 G per tensor) on a duplicated 2048-image batch: both halves' logits must
    match the 2048-image forward (bench.py stays at 2048 img/GPU, every tensor below 2^31 elements; 3072 / 4096
    measured +1.5 / +2.2 % img/s but not adopted: README)."""
    from imagent_amd.models import resnet
    from imagent_amd.models.native import bind_native
    from imagent_amd.ops.misc import normalize_u8
    dev = torch.device(DEV)
    torch.manual_seed(0)
    m = resnet.resnet50()
    bind_native(m, dev)
    m.train()
    img = torch.randint(0, 256, (2048, 224, 224, 3), dtype=torch.uint8, device=dev)
    mean, std = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)
    with torch.no_grad():
        l1 = m(normalize_u8(img, (224, 224), 4, mean, std)).float()
        l2 = m(normalize_u8(torch.cat([img, img]), (224, 224), 4, mean, std)).float()
    assert torch.isfinite(l2).all()
    assert rel(l2[:2048], l1) < 2e-2 and rel(l2[2048:], l1) < 2e-2, (rel(l2[:2048], l1), rel(l2[2048:], l1))


def test_train_step_4096_duplicated_halves():
    """A TRAINING step (forward with batch statistics + backward) at 4096 img on a duplicated 2048-image batch, on a
    bottleneck net with the whole stem and layer 1 (blocks [3, 1, 1, 1]): the stem output and the 256-channel layer-1
    tensors hold 3.3 G elements (6.6 GB: past 2^31 elements and past the 32-bit byte range of one buffer descriptor).
    With both halves identical, every per-pixel kernel sees identical per-channel constants (BatchNorm statistics and
    backward reductions are over the whole batch), so the logits and the gradient flowing into EVERY block input must
    be the same in both halves, bit for bit: any 32-bit element / byte index that wraps shows up as a mismatch. The
    weight gradients (reductions) must equal the 2048-image step's up to summation order: compared with the
    2048-vs-2048 rerun (the float-atomic noise floor)."""
    from imagent_amd.models import resnet
    from imagent_amd.models.native import bind_native
    from imagent_amd.ops import block as blk
    from imagent_amd.ops.misc import XentFn, normalize_u8
    dev = torch.device(DEV)
    torch.manual_seed(0)
    m = resnet.ResNet(resnet.Bottleneck, [3, 1, 1, 1])
    st = bind_native(m, dev)
    m.train()
    B = 2048
    img = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, device=dev)
    lab = torch.randint(0, 1000, (B,), device=dev)
    mean, std = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)
    halves = []
    orig = blk.BlockFn.apply

    def apply(y, b):
        if y.requires_grad and y.shape[0] == 2 * B:
            y.register_hook(lambda g, n=len(halves): halves.append((n, tuple(g.shape), int((g[:B] != g[B:]).sum()))))
        return orig(y, b)

    def step(images, labels):
        st.arena.G.zero_()
        met = torch.zeros(4, device=dev)
        logits = m(normalize_u8(images, (224, 224), 4, mean, std))
        loss = XentFn.apply(logits, labels, met, 0.0)
        loss.backward()
        torch.cuda.synchronize()
        return logits.detach(), st.arena.G.clone()

    _, g1 = step(img, lab)
    _, g1b = step(img, lab)
    blk.BlockFn.apply = apply
    try:
        logits2, g2 = step(torch.cat([img, img]), torch.cat([lab, lab]))
    finally:
        del blk.BlockFn.apply  # back to the inherited torch.autograd.Function.apply
    assert torch.isfinite(logits2).all()
    assert torch.equal(logits2[:B], logits2[B:]), "forward: the two halves differ"
    assert len(halves) == 6, halves
    assert all(bad == 0 for _, _, bad in halves), halves
    # weight gradients: the duplicated step vs the 2048 step, against the 2048-vs-2048 noise floor, per tensor
    ar = st.arena
    worst = 0.0
    for i, name in enumerate(ar.names):
        a, b, c = ar.flat_slice(g2, i), ar.flat_slice(g1, i), ar.flat_slice(g1b, i)
        floor = rel(c, b)
        worst = max(worst, rel(a, b) / max(floor, 1e-4))
    assert worst < 10.0, worst
