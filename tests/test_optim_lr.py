"""Optimizers, LR schedule and meters (imagenet.py:44-94, 154-162, 325-340)."""

import pytest
import torch

from imagent_amd.models.arena import ParamArena
from imagent_amd.train import lr as lrmod
from imagent_amd.train.meters import AverageMeter, DeviceMetrics, accuracy
from imagent_amd.train.optim import FlatSGD, build_optimizer


def _params():
    torch.manual_seed(0)
    a = torch.nn.Parameter(torch.randn(5, 3, 3, 3).contiguous(memory_format=torch.channels_last))
    b = torch.nn.Parameter(torch.randn(7))
    return [("w", a), ("b", b)]


@pytest.mark.parametrize("nesterov,damp", [(False, 0.0), (True, 0.0), (False, 0.3)])
def test_flat_sgd_matches_torch(nesterov, damp):
    named = _params()
    ref = [torch.nn.Parameter(p.detach().clone()) for _, p in named]
    ar = ParamArena(named, "cpu", order=[1, 0])
    opt = FlatSGD(ar, 0.1, momentum=0.9, dampening=damp, weight_decay=1e-4, nesterov=nesterov)
    ropt = torch.optim.SGD(ref, lr=0.1, momentum=0.9, dampening=damp, weight_decay=1e-4, nesterov=nesterov)
    for step in range(4):
        grads = [torch.randn_like(r) for r in ref]
        opt.zero_grad()
        for (_, p), g in zip(named, grads):
            p.grad.add_(g)        # grads live in the arena
        for r, g in zip(ref, grads):
            r.grad = g.clone()
        opt.step()
        ropt.step()
    for (_, p), r in zip(named, ref):
        torch.testing.assert_close(p.detach(), r.detach(), rtol=1e-6, atol=1e-6)


def test_arena_layout_is_channels_last_and_aliased():
    named = _params()
    ar = ParamArena(named, "cpu")
    w = named[0][1]
    assert w.is_contiguous(memory_format=torch.channels_last)
    assert w.data_ptr() == ar.P[ar.offsets[0]:].data_ptr()
    ar.P.fill_(2.0)
    assert float(w.sum()) == 2.0 * w.numel()
    assert ar.offsets[1] % 64 == 0


def test_torch_optimizers_over_arena():
    for name in ["adam", "adamw", "adagrad", "rmsprop", "adadelta", "asgd", "nadam"]:
        named = _params()
        ar = ParamArena(named, "cpu")
        opt = build_optimizer(name, ar, 0.01)
        before = ar.P.clone()
        for _, p in named:
            p.grad.normal_()
        opt.step()
        assert not torch.equal(before, ar.P), name
    with pytest.raises(ValueError):
        build_optimizer("fr", ParamArena(_params(), "cpu"), 0.1)


def test_reference_lr_schedule():
    assert lrmod.step_lr(0.1, 0) == 0.1
    assert lrmod.step_lr(0.1, 29) == 0.1
    assert abs(lrmod.step_lr(0.1, 30) - 0.01) < 1e-12      # imagent_sgd.out:454
    assert abs(lrmod.step_lr(0.1, 60) - 0.001) < 1e-12
    assert abs(lrmod.step_lr(0.1, 99) - 1e-4) < 1e-12
    s = lrmod.Schedule(0.1, 90, 100, warmup_epochs=5, scale_batch=8192)
    assert abs(s(0, 0) - 3.2 / 500) < 1e-9
    assert abs(s(5, 0) - 3.2) < 1e-9
    c = lrmod.Schedule(0.1, 10, 10, kind="cosine")
    assert abs(c(0) - 0.1) < 1e-9 and c(9, 9) < 0.01


def test_meters_and_accuracy():
    m = AverageMeter()
    m.update(2.0, 3)
    m.update(4.0, 1)
    assert m.avg == 2.5 and m.count == 4
    out = torch.tensor([[0.1, 0.9, 0.0, 0.0, 0.0, 0.0], [0.9, 0.05, 0.04, 0.01, 0.0, 0.0]])
    t = torch.tensor([1, 3])
    p1, p5 = accuracy(out, t, (1, 5))
    assert p1.item() == 50.0 and p5.item() == 100.0
    dm = DeviceMetrics("cpu")
    dm.update_from_logits(out, t, torch.tensor(1.5))
    loss, t1, t5, n = dm.reduced()
    assert (loss, t1, t5, n) == (1.5, 50.0, 100.0, 2.0)


def test_lars_matches_reference_math():
    """FlatLARS (CPU path) vs a direct per-parameter LARS reference, 3 steps."""
    import torch.nn as nn

    from imagent_amd.models.arena import ParamArena
    from imagent_amd.train.optim import FlatLARS
    torch.manual_seed(0)
    net = nn.Sequential(nn.Conv2d(3, 8, 3), nn.BatchNorm2d(8))
    ref = [p.detach().clone() for p in net.parameters()]
    ar = ParamArena(list(net.named_parameters()), torch.device("cpu"))
    opt = FlatLARS(ar, lr=0.5, momentum=0.9, weight_decay=1e-4, eta=1e-3, native=False)
    vel = [torch.zeros_like(p) for p in ref]
    for step in range(3):
        grads = [torch.randn_like(p) for p in ref]
        for p, g in zip(net.parameters(), grads):
            p.grad.copy_(g)
        opt.step()
        for i, (w, g) in enumerate(zip(ref, grads)):
            adapt = w.dim() > 1
            wd = 1e-4 if adapt else 0.0
            trust = 1e-3 * w.norm() / (g.norm() + 1e-4 * w.norm()) if adapt else 1.0
            d = g + wd * w
            vel[i] = 0.5 * trust * d if step == 0 else 0.9 * vel[i] + 0.5 * trust * d
            w -= vel[i]
    for p, w in zip(net.parameters(), ref):
        assert torch.allclose(p.detach(), w, rtol=1e-5, atol=1e-6)
