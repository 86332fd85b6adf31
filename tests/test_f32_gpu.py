"""fp32 kernel path (csrc/kernels/f32.hip, ops/f32.py, models/native_f32.py) against PyTorch.

The reference trains in fp32 (imagenet.py:312, no AMP). Every fp32 op is checked two ways: within
1e-4 relative (normwise) of the PyTorch fp32 op, and no farther from the float64 result than 4x
PyTorch fp32's own distance to it (+1e-6) -- i.e. as accurate as the PyTorch fp32 path, not just
close to it. The whole-model test runs two ResNet-18 training steps against float64.
"""

import os
import sys

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
DEV = "cuda"
TOL = 1e-4


def rel(a, b):
    a, b = a.detach(), b.detach()
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


def as_good(ours, torch32, exact, floor=1e-6):
    """ours within 1e-4 of torch fp32 and as close to float64 as torch fp32 is (4x, + floor)."""
    return rel(ours, torch32) < TOL and rel(ours, exact) <= 4 * rel(torch32, exact) + floor


def nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


def nchw(t):
    return t.permute(0, 3, 1, 2)


@pytest.fixture(autouse=True)
def _no_tf32():
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False


@pytest.mark.parametrize("shape", [(4, 64, 14, 128, 3, 1, 1), (3, 72, 11, 200, 3, 2, 1), (2, 256, 9, 512, 1, 1, 0),
                                   (2, 128, 15, 64, 1, 2, 0), (3, 4, 38, 64, 7, 2, 3), (2, 64, 57, 64, 3, 1, 1),
                                   (5, 96, 7, 40, 1, 1, 0)])
def test_conv_f32_fwd_dgrad_wgrad(shape):
    from imagent_amd.ops.f32 import conv_f32, dgrad_f32, wgrad_f32
    N, Ci, H, Co, k, s, p = shape
    torch.manual_seed(0)
    x = torch.randn(N, Ci, H, H, device=DEV, requires_grad=True)
    w = (torch.randn(Co, Ci, k, k, device=DEV) * (2.0 / (Ci * k * k)) ** 0.5).requires_grad_(True)
    y = F.conv2d(x, w, None, s, p)
    g = torch.randn_like(y)
    y.backward(g)
    x64 = x.detach().double().requires_grad_(True)
    w64 = w.detach().double().requires_grad_(True)
    y64 = F.conv2d(x64, w64, None, s, p)
    y64.backward(g.double())
    wk = w.detach().permute(0, 2, 3, 1).contiguous()
    got = conv_f32(nhwc(x.detach()), wk, s, p, k, k)
    assert as_good(nchw(got), y, y64)
    dx = dgrad_f32(nhwc(g), wk.permute(3, 1, 2, 0).contiguous(), (H, H), s, p, k, k)
    assert as_good(nchw(dx), x.grad, x64.grad)
    dw = torch.zeros(Co, k, k, Ci, device=DEV)
    wgrad_f32(nhwc(g), nhwc(x.detach()), dw, s, p, k, k)
    assert as_good(dw.permute(0, 3, 1, 2), w.grad, w64.grad)


@pytest.mark.parametrize("shape", [(4, 64, 14, 128, 3, 1, 1), (3, 72, 11, 200, 3, 2, 1), (2, 256, 9, 512, 1, 1, 0),
                                   (3, 4, 38, 64, 7, 2, 3), (2, 64, 57, 64, 3, 1, 1), (5, 96, 7, 40, 1, 1, 0)])
def test_conv_f32_split(shape):
    """The 3 x bf16 split forward / dgrad / wgrad (f32.hip igemm_f32s_kernel, wgrad_f32s_kernel,
    ops.f32.set_split): within 1e-4 of the PyTorch fp32 conv (normwise) -- ~2^-16 per product, not the exact
    kernels' as-good-as-fp32 bound."""
    from imagent_amd.ops.f32 import conv_f32, dgrad_f32, set_split, wgrad_f32
    N, Ci, H, Co, k, s, p = shape
    torch.manual_seed(0)
    x = torch.randn(N, Ci, H, H, device=DEV, requires_grad=True)
    w = (torch.randn(Co, Ci, k, k, device=DEV) * (2.0 / (Ci * k * k)) ** 0.5).requires_grad_(True)
    y = F.conv2d(x, w, None, s, p)
    g = torch.randn_like(y)
    y.backward(g)
    wk = w.detach().permute(0, 2, 3, 1).contiguous()
    set_split(True)
    try:
        got = conv_f32(nhwc(x.detach()), wk, s, p, k, k)
        dx = dgrad_f32(nhwc(g), wk.permute(3, 1, 2, 0).contiguous(), (H, H), s, p, k, k)
        dw = torch.zeros(Co, k, k, Ci, device=DEV)
        wgrad_f32(nhwc(g), nhwc(x.detach()), dw, s, p, k, k)
        torch.cuda.synchronize()
    finally:
        set_split(False)
    assert rel(nchw(got), y) < TOL, rel(nchw(got), y)
    assert rel(nchw(dx), x.grad) < TOL, rel(nchw(dx), x.grad)
    assert rel(dw.permute(0, 3, 1, 2), w.grad) < TOL, rel(dw.permute(0, 3, 1, 2), w.grad)


@pytest.mark.parametrize("C,res,relu", [(64, False, True), (128, True, True), (256, False, False), (512, True, True),
                                        (1024, False, True), (2048, True, True)])
def test_bn_f32(C, res, relu):
    from imagent_amd.models.resnet import BatchNorm2d
    from imagent_amd.ops.f32 import BNF32Fn, F32Workspace
    torch.manual_seed(1)
    N, H = 6, 9
    x = (torch.randn(N, C, H, H, device=DEV) * 3 + 5).requires_grad_(True)
    r = torch.randn(N, C, H, H, device=DEV, requires_grad=True) if res else None
    bn = BatchNorm2d(C).to(DEV)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    bn.weight.grad = torch.zeros_like(bn.weight)
    bn.bias.grad = torch.zeros_like(bn.bias)
    rm, rv = bn.running_mean.clone(), bn.running_var.clone()  # reference running stats
    F.batch_norm(x.detach(), rm, rv, None, None, True, 0.1, 1e-5)
    gam = bn.weight.detach().clone().requires_grad_(True)
    bet = bn.bias.detach().clone().requires_grad_(True)
    yr = F.batch_norm(x, bn.running_mean.clone(), bn.running_var.clone(), gam, bet, True, 0.1, 1e-5)
    if res:
        yr = yr + r
    if relu:
        yr = F.relu(yr)
    g = torch.randn_like(yr)
    yr.backward(g)
    x64 = x.detach().double().requires_grad_(True)
    r64 = r.detach().double().requires_grad_(True) if res else None
    g64_, b64_ = gam.detach().double().requires_grad_(True), bet.detach().double().requires_grad_(True)
    y64 = F.batch_norm(x64, None, None, g64_, b64_, True, 0.1, 1e-5)
    if res:
        y64 = y64 + r64
    if relu:
        y64 = F.relu(y64)
    y64.backward(g.double())
    ws = F32Workspace(DEV, C)
    xn = nhwc(x.detach()).requires_grad_(True)
    rn = nhwc(r.detach()).requires_grad_(True) if res else None
    y = BNF32Fn.apply(xn, rn, bn, relu, ws)
    assert as_good(nchw(y), yr, y64)
    assert rel(bn.running_mean, rm) < TOL and rel(bn.running_var, rv) < TOL
    y.backward(nhwc(g))
    assert as_good(nchw(xn.grad), x.grad, x64.grad)
    assert as_good(bn.weight.grad, gam.grad, g64_.grad) and as_good(bn.bias.grad, bet.grad, b64_.grad)
    if res:
        assert as_good(nchw(rn.grad), r.grad, r64.grad)


def test_pool_fc_xent_f32():
    from imagent_amd.ops.f32 import AvgPoolF32Fn, MaxPoolF32Fn, XentF32Fn
    torch.manual_seed(2)
    x = torch.randn(3, 16, 17, 17, device=DEV, requires_grad=True)
    y = F.max_pool2d(x, 3, 2, 1)
    g = torch.randn_like(y)
    y.backward(g)
    xn = nhwc(x.detach()).requires_grad_(True)
    yn = MaxPoolF32Fn.apply(xn, 3, 2, 1)
    assert rel(nchw(yn), y.detach()) < TOL
    yn.backward(nhwc(g))
    assert rel(nchw(xn.grad), x.grad) < TOL
    a = torch.randn(4, 7, 7, 32, device=DEV, requires_grad=True)
    pa = AvgPoolF32Fn.apply(a)
    assert rel(pa, a.detach().mean((1, 2))) < TOL
    z = torch.randn(8, 1000, device=DEV, requires_grad=True)
    lab = torch.randint(0, 1000, (8,), device=DEV)
    met = torch.zeros(4, device=DEV)
    loss = XentF32Fn.apply(z, lab, met, 0.0)
    zr = z.detach().clone().requires_grad_(True)
    lr_ = F.cross_entropy(zr, lab)
    lr_.backward()
    loss.backward()
    assert abs(loss.item() - lr_.item()) < 1e-5
    assert rel(z.grad, zr.grad) < TOL


@pytest.mark.parametrize("split", [False, True])
def test_resnet18_f32_training_step_matches_torch(split):
    """Two full training steps (normalise -> forward -> xent -> backward -> SGD) of ResNet-18 on the
    fp32 kernels against the same model in float64 (PyTorch ops). The first forward (loss) is within
    1e-4 relative; what depends on the gradients (updated parameters, the second loss, eval logits)
    within 3x PyTorch fp32's own distance to float64, or 2e-3.

    Gradients get a looser 1e-2 bound, because of the ReLU: an activation within rounding of 0 can
    take the other side of the mask in ANY fp32 forward, and one such flip among ~10^5 activations
    moves that BatchNorm's bias gradient (a sum that cancels to ~5 % of its terms) by ~2e-3 and
    every gradient below it by as much (scripts/f32_diag.py: one flip at layer3.1.bn1 gives exactly
    the 1-3e-3 seen at every earlier layer, with the same gradients computed under float64's mask
    matching to 2.5e-6; PyTorch fp32 flips too on other seeds, 4.5e-3 at layer1.1.bn2.bias).
    ``split``: every conv on the 3 x bf16 split kernels (bench.py --fp32-split). ~2^-16 per product puts
    ~10x more activations within rounding of the ReLU threshold, so the flip-driven gradient floor is
    4e-2 (measured 1.0-1.5e-2 at the first layers) -- still tighter than the TF32 convs PyTorch runs
    fp32 models on by default on the reference's GPUs (10-bit mantissa, 2^-11 per product).

    In both modes the oracles restart step 2 from OUR state (weights, BatchNorm statistics, momentum): after
    the lr-0.1 step on 8 images (loss 4.74 -> 2.75) the step-2 gradients amplify a step-1 gradient difference
    ~40-100x (measured: split 1e-2 -> 0.4; exact, on a run where one ReLU flip gave 2e-3, -> 0.2, with
    PyTorch fp32's own step-1 flip at 2.3e-3), so oracles that kept their own weights test the chaos, not
    the kernels.
    """
    from imagent_amd.ops.f32 import set_split
    set_split(split)
    try:
        _r18_f32_steps(4e-2 if split else 1e-2, True)
    finally:
        set_split(False)


def test_resnet50_f32_forward_backward_matches_float64():
    """ResNet-50 on the fp32 kernels (2048-channel BatchNorms: two 1024-channel statistics slices):
    one forward + backward on 4 images against the same model in float64. Loss within 1e-4;
    gradients within 3x PyTorch fp32's own distance to float64 or 1e-2 (ReLU flips, see the ResNet-18
    test)."""
    import copy
    from imagent_amd.data.loader import InputTransform
    from imagent_amd.models import resnet
    from imagent_amd.models.native_f32 import bind_native_f32
    from imagent_amd.ops.f32 import XentF32Fn
    torch.manual_seed(5)
    ref = resnet.resnet50(num_classes=100).to(DEV)
    ref64 = copy.deepcopy(ref).double()
    m = resnet.resnet50(num_classes=100)
    m.load_state_dict(ref.state_dict())
    st = bind_native_f32(m, DEV)
    u8 = torch.randint(0, 256, (4, 64, 64, 3), dtype=torch.uint8, device=DEV)
    y = torch.randint(0, 100, (4,), device=DEV)
    xr = InputTransform("torch", (64, 64))(u8)
    xh = InputTransform("hip_f32", (64, 64), cpad=4)(u8)
    for mm in (ref, ref64, m):
        mm.train()
    st.arena.zero_grad()
    l32 = F.cross_entropy(ref(xr), y)
    l32.backward()
    l64 = F.cross_entropy(ref64(xr.double()), y)
    l64.backward()
    met = torch.zeros(4, device=DEV)
    loss = XentF32Fn.apply(m(xh), y, met, 0.0)
    loss.backward()
    torch.cuda.synchronize()
    assert abs(loss.item() - l64.item()) < 1e-4 * max(1.0, abs(l64.item())), (loss.item(), l64.item())
    g32 = {n: p.grad for n, p in ref.named_parameters()}
    g64 = {n: p.grad for n, p in ref64.named_parameters()}
    bad = [(n, f"{rel(p.grad, g64[n]):.2e}", f"{rel(g32[n], g64[n]):.2e}") for n, p in m.named_parameters()
           if not rel(p.grad, g64[n]) <= max(3 * rel(g32[n], g64[n]), 1e-2)]
    assert not bad, bad


@pytest.mark.parametrize("split", [True, False])
@pytest.mark.parametrize("arch", ["resnet18", "resnet50"])
def test_f32_block_node_matches_per_op(arch, split):
    """BlockF32Fn (one autograd node per residual block: conv1's dgrad accumulates the residual gradient in
    its epilogue, weight gradients on the side stream) against the per-op autograd nodes on the same weights
    and input: loss, every gradient and the BatchNorm buffers. Deterministic mode, so both paths take the
    fixed-order statistics passes and the comparison is exact up to fp32 add order (1e-5)."""
    import copy
    from imagent_amd.data.loader import InputTransform
    from imagent_amd.models import resnet
    from imagent_amd.models.native_f32 import bind_native_f32
    from imagent_amd.ops.conv import set_deterministic
    from imagent_amd.ops.f32 import XentF32Fn, set_split
    torch.manual_seed(9)
    base = getattr(resnet, arch)(num_classes=100)
    u8 = torch.randint(0, 256, (4, 64, 64, 3), dtype=torch.uint8, device=DEV)
    y = torch.randint(0, 100, (4,), device=DEV)
    xh = InputTransform("hip_f32", (64, 64), cpad=4)(u8)
    out = []
    set_deterministic(True)
    set_split(split)
    try:
        for fused in (True, False):
            m = copy.deepcopy(base)
            st = bind_native_f32(m, DEV)
            st.fused_blocks = fused
            m.train()
            st.arena.zero_grad()
            loss = XentF32Fn.apply(m(xh), y, torch.zeros(4, device=DEV), 0.0)
            loss.backward()
            torch.cuda.synchronize()
            out.append((loss.item(), {n: p.grad.clone() for n, p in m.named_parameters()},
                        {n: b.clone() for n, b in m.named_buffers()}))
    finally:
        set_split(False)
        set_deterministic(False)
    (l1, g1, b1), (l2, g2, b2) = out
    assert abs(l1 - l2) < 1e-6 * max(1.0, abs(l2)), (l1, l2)
    bad = [(n, rel(g1[n], g2[n])) for n in g1 if rel(g1[n], g2[n]) > 1e-5]
    assert not bad, bad
    assert all(rel(b1[n].float(), b2[n].float()) < 1e-6 for n in b1)


def _r18_f32_steps(gfloor, resync):
    import copy
    from imagent_amd.data.loader import InputTransform
    from imagent_amd.models import resnet
    from imagent_amd.models.arena import ParamArena
    from imagent_amd.models.native_f32 import bind_native_f32
    from imagent_amd.ops.f32 import XentF32Fn
    from imagent_amd.train.optim import FlatSGD
    torch.manual_seed(3)
    ref = resnet.resnet18(num_classes=100).to(DEV)
    ref64 = copy.deepcopy(ref).double()
    m = resnet.resnet18(num_classes=100)
    m.load_state_dict(ref.state_dict())
    st = bind_native_f32(m, DEV)
    models = [(ref, ParamArena(list(ref.named_parameters()), torch.device(DEV))),
              (ref64, None), (m, st.arena)]
    opts = [FlatSGD(models[0][1], lr=0.1, momentum=0.9, weight_decay=1e-4),
            torch.optim.SGD(ref64.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4),
            FlatSGD(st.arena, lr=0.1, momentum=0.9, weight_decay=1e-4)]
    u8 = torch.randint(0, 256, (8, 112, 112, 3), dtype=torch.uint8, device=DEV)
    y = torch.randint(0, 100, (8,), device=DEV)
    xr = InputTransform("torch", (112, 112))(u8)
    xh = InputTransform("hip_f32", (112, 112), cpad=4)(u8)
    assert rel(nchw(xh[..., :3]), xr) < 1e-6

    def close(ours, oracle32, exact, floor=1e-4):
        return rel(ours, exact) <= max(3 * rel(oracle32, exact), floor)

    for it in range(2):
        if resync and it:  # weights, BN statistics and momentum buffers from ours
            for mm in (ref, ref64):
                mm.load_state_dict(m.state_dict())
            ours, ra, p64 = st.arena, models[0][1], dict(ref64.named_parameters())
            for i, n in enumerate(ours.names):
                b = ours.view(opts[2].buf, i)
                ra.view(opts[0].buf, ra.names.index(n)).copy_(b)
                opts[1].state[p64[n]]["momentum_buffer"].copy_(b)
        for mm, _ in models:
            mm.train()
        for o in opts:
            o.zero_grad()
        l32 = F.cross_entropy(ref(xr), y)
        l32.backward()
        l64 = F.cross_entropy(ref64(xr.double()), y)
        l64.backward()
        met = torch.zeros(4, device=DEV)
        loss = XentF32Fn.apply(m(xh), y, met, 0.0)
        loss.backward()
        # step 0: the same weights -> 1e-4; step 1 runs on weights updated with those (flip-affected,
        # see above) gradients, lr 0.1: the loss moved 4.74 -> 2.75 and carries their 1e-3 (measured 6e-4)
        ltol = 1e-4 if it == 0 else 2e-3
        assert abs(loss.item() - l64.item()) < ltol * max(1.0, abs(l64.item())), (it, loss.item(), l64.item())
        g32 = {n: p.grad for n, p in ref.named_parameters()}
        g64 = {n: p.grad for n, p in ref64.named_parameters()}
        bad = [(n, f"{rel(p.grad, g64[n]):.2e}", f"{rel(g32[n], g64[n]):.2e}") for n, p in m.named_parameters()
               if not close(p.grad, g32[n], g64[n], gfloor)]
        assert not bad, (it, bad)
        for o in opts:
            o.step()
    # a parameter made of its updates (BatchNorm biases start at 0) inherits the step-2 gradient difference
    # (split: measured 6.4e-3 at layer1.0.bn1.bias) and so gets the gradients' own floor; the others, whose
    # two lr-0.1 updates are a small part of their value, the tighter state floor (exact: one ReLU flip put
    # 2.8e-3 on layer2.1.bn1.bias, a 1e-2-floor gradient's 1e-2 can land there in full)
    sfloor = 1e-2 if gfloor > 1e-2 else 2e-3
    sd32, sd64 = ref.state_dict(), ref64.state_dict()
    zero_init = {n for n, p in ref.named_parameters() if n.endswith(".bias")}
    for n, a in m.state_dict().items():
        if a.dtype.is_floating_point:
            fl = max(sfloor, gfloor) if n in zero_init else sfloor
            assert close(a, sd32[n], sd64[n], fl), (n, rel(a, sd64[n]))
    for mm, _ in models:
        mm.eval()
    with torch.no_grad():
        assert close(m(xh), ref(xr), ref64(xr.double()), sfloor), rel(m(xh), ref64(xr.double()))
