"""fp32 kernel path (csrc/kernels/f32.hip, ops/f32.py, models/native_f32.py) against PyTorch fp32.

The reference trains in fp32 (imagenet.py:312, no AMP): every fp32 op is compared with the
PyTorch fp32 op at <= 1e-4 relative (normwise), and a whole ResNet-18 training step (forward,
backward, SGD) with the fp32 oracle model.
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
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


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
    wk = w.detach().permute(0, 2, 3, 1).contiguous()
    got = conv_f32(nhwc(x.detach()), wk, s, p, k, k)
    assert rel(nchw(got), y.detach()) < TOL
    dx = dgrad_f32(nhwc(g), wk.permute(3, 1, 2, 0).contiguous(), (H, H), s, p, k, k)
    assert rel(nchw(dx), x.grad) < TOL
    dw = torch.zeros(Co, k, k, Ci, device=DEV)
    wgrad_f32(nhwc(g), nhwc(x.detach()), dw, s, p, k, k)
    assert rel(dw.permute(0, 3, 1, 2), w.grad) < TOL


@pytest.mark.parametrize("C,res,relu", [(64, False, True), (128, True, True), (256, False, False), (512, True, True)])
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
    ws = F32Workspace(DEV, C)
    xn = nhwc(x.detach()).requires_grad_(True)
    rn = nhwc(r.detach()).requires_grad_(True) if res else None
    y = BNF32Fn.apply(xn, rn, bn, relu, ws)
    assert rel(nchw(y), yr.detach()) < TOL
    assert rel(bn.running_mean, rm) < TOL and rel(bn.running_var, rv) < TOL
    y.backward(nhwc(g))
    assert rel(nchw(xn.grad), x.grad) < TOL
    assert rel(bn.weight.grad, gam.grad) < TOL and rel(bn.bias.grad, bet.grad) < TOL
    if res:
        assert rel(nchw(rn.grad), r.grad) < TOL


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


def test_resnet18_f32_training_step_matches_torch():
    """One full training step (normalise -> forward -> xent -> backward -> SGD) of ResNet-18 on the
    fp32 kernels against the same model on PyTorch fp32 ops."""
    from imagent_amd.data.loader import InputTransform
    from imagent_amd.models import resnet
    from imagent_amd.models.arena import ParamArena
    from imagent_amd.models.native_f32 import bind_native_f32
    from imagent_amd.ops.f32 import XentF32Fn
    from imagent_amd.train.optim import FlatSGD
    torch.manual_seed(3)
    ref = resnet.resnet18(num_classes=100).to(DEV)
    m = resnet.resnet18(num_classes=100)
    m.load_state_dict(ref.state_dict())
    st = bind_native_f32(m, DEV)
    ar = ParamArena(list(ref.named_parameters()), torch.device(DEV))
    opt_r = FlatSGD(ar, lr=0.1, momentum=0.9, weight_decay=1e-4)
    opt = FlatSGD(st.arena, lr=0.1, momentum=0.9, weight_decay=1e-4)
    u8 = torch.randint(0, 256, (8, 64, 64, 3), dtype=torch.uint8, device=DEV)
    y = torch.randint(0, 100, (8,), device=DEV)
    xr = InputTransform("torch", (64, 64))(u8)
    xh = InputTransform("hip_f32", (64, 64), cpad=4)(u8)
    assert rel(nchw(xh[..., :3]), xr) < 1e-6
    for it in range(2):
        ref.train()
        m.train()
        opt_r.zero_grad()
        opt.zero_grad()
        lr_ = F.cross_entropy(ref(xr), y)
        lr_.backward()
        met = torch.zeros(4, device=DEV)
        loss = XentF32Fn.apply(m(xh), y, met, 0.0)
        loss.backward()
        assert abs(loss.item() - lr_.item()) < 1e-4 * max(1.0, abs(lr_.item())), (it, loss.item(), lr_.item())
        gr = {n: p.grad for n, p in ref.named_parameters()}
        for n, p in m.named_parameters():
            assert rel(p.grad, gr[n]) < 1e-3, (it, n, rel(p.grad, gr[n]))
        opt_r.step()
        opt.step()
    for (n, a), (_, b) in zip(m.state_dict().items(), ref.state_dict().items()):
        if a.dtype.is_floating_point:
            assert rel(a, b) < 1e-4, n
    m.eval()
    ref.eval()
    with torch.no_grad():
        assert rel(m(xh), ref(xr)) < 1e-4
