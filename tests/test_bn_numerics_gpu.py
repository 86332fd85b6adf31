"""BatchNorm batch statistics when |mean| >> std.

The conv epilogue accumulates per-channel sums of ``v - shift`` and
``(v - shift)^2`` with shift = the BN's previous batch mean (``work.save``),
and the finalize kernel returns (mean, biased variance). Raw sum / sum of
squares in fp32 (E[x^2] - mean^2) loses the variance when |mean|/std ~ 100.
Reference semantics: ``torch.nn.BatchNorm2d`` training statistics
(imagenet.py:312); checked against fp64 over the bf16 values the BN reads.
"""

import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
DEV = "cuda"


def _work(C):
    from imagent_amd.models.resnet import BNWork
    from imagent_amd.ops import _lib
    return BNWork(torch.zeros(_lib.STAT_SLOTS, 2, C, device=DEV), torch.zeros(2, C, device=DEV),
                  torch.zeros(2, C, device=DEV), torch.zeros(_lib.kernels().imk_bn_bwd_scratch_floats(C), device=DEV))


@pytest.mark.parametrize("Co", [64, 256])
def test_shifted_statistics_large_mean(Co):
    from imagent_amd.ops.bn import stats_finalize
    from imagent_amd.ops.conv import igemm_fwd
    torch.manual_seed(0)
    N, H, Ci = 1000, 32, 64            # R = 1,024,000 rows per channel
    x = torch.randn(N, H, H, Ci, device=DEV)
    x[..., -1] = 1.0                    # a constant input channel carries the large mean
    w = torch.randn(Co, 1, 1, Ci, device=DEV) * 0.1
    w[..., -1] = 100.0 + torch.rand(Co, 1, 1, device=DEV)  # mean ~100, std ~0.8: |mean|/std > 100
    x, w = x.to(torch.bfloat16), w.to(torch.bfloat16)
    work = _work(Co)
    R = N * H * H
    errs = []
    for call in range(2):
        work.slab.zero_()
        y = igemm_fwd(x, w, 1, 0, 1, 1, stats=work)
        stats_finalize(work, R)
        yd = y.double().reshape(-1, Co)
        mean64, var64 = yd.mean(0), yd.var(0, unbiased=False)
        assert float((mean64.abs() / var64.sqrt()).min()) > 100.0
        mean, var = work.stats[0].double(), work.stats[1].double()
        errs.append((float(((mean - mean64).abs() / var64.sqrt()).max()),
                     float(((var - var64).abs() / var64).max())))
        work.save[0].copy_(work.stats[0])  # what bn_fwd stores: this batch's mean = next shift
    # call 0 runs with shift 0 (fresh BN): E[x^2] - mean^2 in fp32 -- printed for contrast only
    print(f"Co={Co}: shift 0 -> mean err {errs[0][0]:.2e} sd, var rel err {errs[0][1]:.2e}; "
          f"shifted -> mean err {errs[1][0]:.2e} sd, var rel err {errs[1][1]:.2e}")
    assert errs[1][0] < 1e-3, errs
    assert errs[1][1] < 1e-3, errs


@pytest.mark.parametrize("mode", [1, 2])
def test_bn_fwd_relu_mask_bits(mode):
    """bn_fwd's ReLU-mask bit output (ym) equals (y > 0) of the bf16 output it stores, packed as
    ops.bn.relu_mask_bits -- the mask the next block's conv1 dgrad epilogue reads instead of y."""
    from imagent_amd.models.resnet import BatchNorm2d
    from imagent_amd.ops.bn import bn_fwd_launch, relu_mask_bits
    torch.manual_seed(1)
    N, H, C = 8, 14, 256
    x = torch.randn(N, H, H, C, device=DEV).to(torch.bfloat16)
    x2 = torch.randn(N, H, H, C, device=DEV).to(torch.bfloat16)
    bn, bn2 = BatchNorm2d(C).to(DEV), BatchNorm2d(C).to(DEV)
    stats = torch.stack([torch.randn(C, device=DEV) * 0.1, torch.rand(C, device=DEV) + 0.5])
    stats2 = torch.stack([torch.randn(C, device=DEV) * 0.1, torch.rand(C, device=DEV) + 0.5])
    y = torch.empty_like(x)
    ym = torch.full((x.numel() // 8,), 0xA5, device=DEV, dtype=torch.uint8)
    kw = dict(stats2=stats2, gamma2=bn2.weight, beta2=bn2.bias) if mode == 2 else {}
    bn_fwd_launch(x, stats, bn.weight, bn.bias, y, None, x2=x2, mode=mode, relu=True, ym=ym, **kw)
    torch.cuda.synchronize()
    assert (y > 0).any() and (y == 0).any()
    assert torch.equal(ym, relu_mask_bits(y))


def test_deterministic_statistics():
    """Deterministic mode: the conv's forward statistics come from the fixed-order pass over its output
    (bn.hip bn_stats_det_kernel + det_fold_kernel): bit-identical across runs, equal to the epilogue
    statistics and to fp64 over the stored bf16 output within fp32 rounding; the BN-backward reduce pass
    with the fixed-order fold gives bit-identical dx / reductions across runs."""
    from imagent_amd.models.resnet import BatchNorm2d
    from imagent_amd.ops import conv as cv
    from imagent_amd.ops.bn import bn_act_backward, stats_finalize
    torch.manual_seed(5)
    N, H, Ci, Co = 64, 28, 128, 256
    x = torch.randn(N, H, H, Ci, device=DEV).to(torch.bfloat16)
    w = (torch.randn(Co, 3, 3, Ci, device=DEV) * 0.05).to(torch.bfloat16)
    shift = torch.randn(Co, device=DEV) * 0.1
    prev = cv.deterministic()

    def fwd(det):
        work = _work(Co)
        work.save[0].copy_(shift)
        cv.set_deterministic(det)
        try:
            y = cv.igemm_fwd(x, w, 1, 1, 3, 3, stats=work)
            stats_finalize(work, y.numel() // Co)
        finally:
            cv.set_deterministic(prev)
        torch.cuda.synchronize()
        return y, work.stats.clone()

    y0, s0 = fwd(False)
    y1, s1 = fwd(True)
    y2, s2 = fwd(True)
    assert torch.equal(y1, y2) and torch.equal(y0, y1)
    assert torch.equal(s1, s2)
    yd = y1.double().reshape(-1, Co)
    mean, var = yd.mean(0), yd.var(0, unbiased=False)
    for s in (s0, s1):
        assert ((s[0].double() - mean).abs() / (var.sqrt() + 1e-6)).max() < 1e-5
        assert ((s[1].double() - var).abs() / var).max() < 1e-4
    # backward reduce + apply, twice in the deterministic mode
    bn = BatchNorm2d(Co).to(DEV)
    bn.work = _work(Co)
    bn.work.save.copy_(torch.stack([mean.float(), torch.rsqrt(var.float() + 1e-5)]))
    bn.weight.grad = torch.zeros_like(bn.weight)
    bn.bias.grad = torch.zeros_like(bn.bias)
    g = torch.randn(N, H, H, Co, device=DEV).to(torch.bfloat16)
    outs = []
    cv.set_deterministic(True)
    try:
        for _ in range(2):
            bn.work.scratch.zero_()
            dx, _ = bn_act_backward(g, y1, None, None, bn, None, 0, True)
            torch.cuda.synchronize()
            outs.append((dx.clone(), bn.work.scratch.clone()))
    finally:
        cv.set_deterministic(prev)
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


class _NS:
    def __init__(self, **kw):
        self.__dict__.update(kw)


@pytest.mark.parametrize("p,sig", [(64, 0.2), (128, 0.3), (256, 0.3), (128, 0.1)])
def test_gram_statistics_large_mean(p, sig):
    """bn3's statistics in the Gram form (ops/bn_gram.py gram_fwd_stats: x3 = h2 W3^T never formed) and on the
    per-op path (conv epilogue, shifted sums) when |mean(x3)| / std(x3) >= 30 (>= 100 with sig = 0.1; |mean| / std ~
    sqrt(p) / sig): half of conv3's output channels
    have weight rows aligned with the (positive, ReLU-like) mean of h2. Checked against fp64 statistics of
    h2 W3^T over the same bf16 operands: mean to 1e-3 sd, variance to 1e-3 relative. Also the x-free backward
    coefficient sum(g xhat3) (bn_bwd_coef_T_kernel: from T = g^T h2, centred per element) against fp64."""
    from imagent_amd.ops import _lib
    from imagent_amd.ops.bn import stats_finalize
    from imagent_amd.ops.bn_gram import gram_T, gram_coef, gram_fwd_stats
    from imagent_amd.ops.conv import colsum_into, igemm_fwd
    torch.manual_seed(7)
    N, H, C4 = 256, 32, 4 * p
    M = N * H * H
    h2 = (1.0 + sig * torch.randn(N, H, H, p, device=DEV)).clamp_min(0).to(torch.bfloat16)
    w = torch.randn(C4, p, device=DEV) / p ** 0.5
    w[: C4 // 2] = (1.0 + 0.1 * torch.randn(C4 // 2, p, device=DEV)) / p  # aligned rows: mean ~1, std ~0.3/sqrt(p)
    w3 = w.to(torch.bfloat16)
    x3 = h2.reshape(M, p).double() @ w3.double().t()
    mean64, var64 = x3.mean(0), x3.var(0, unbiased=False)
    sd64 = var64.sqrt()
    assert float((mean64[: C4 // 2].abs() / sd64[: C4 // 2]).min()) >= (100.0 if sig < 0.2 else 30.0)
    bn = _NS(work=_work(C4), weight=torch.rand(C4, device=DEV) + 0.5, bias=torch.randn(C4, device=DEV) * 0.1,
             eps=1e-5)
    conv = _NS(out_channels=C4, in_channels=p, w_bf16=w3.view(C4, 1, 1, p))
    s = torch.zeros(p, device=DEV)
    colsum_into(h2.view(-1, p), s)
    G = torch.zeros(p, p, device=DEV)
    gram_fwd_stats(bn, conv, h2, s, G)
    torch.cuda.synchronize()
    mean, var = bn.work.stats[0].double(), bn.work.stats[1].double()
    e_mean = float(((mean - mean64).abs() / sd64).max())
    e_var = float(((var - var64).abs() / var64).max())
    print(f"p={p} sig={sig}: Gram form mean err {e_mean:.2e} sd, var rel err {e_var:.2e}")
    assert e_mean < 1e-3 and e_var < 1e-3
    # per-op path: the conv epilogue's shifted sums over the stored bf16 x3 (second call: shift = first mean)
    work = _work(C4)
    for _ in range(2):
        work.slab.zero_()
        y = igemm_fwd(h2, conv.w_bf16, 1, 0, 1, 1, stats=work)
        stats_finalize(work, M)
        work.save[0].copy_(work.stats[0])
    yd = y.double().reshape(-1, C4)
    ym, yv = yd.mean(0), yd.var(0, unbiased=False)
    pe_mean = float(((work.stats[0].double() - ym).abs() / yv.sqrt()).max())
    pe_var = float(((work.stats[1].double() - yv).abs() / yv).max())
    print(f"p={p}: per-op path mean err {pe_mean:.2e} sd, var rel err {pe_var:.2e}")
    assert pe_mean < 1e-3 and pe_var < 1e-3
    # x-free backward coefficient: g correlated with xhat3, nonzero mean (sum(g) ~ M / 2)
    xhat = (x3 - mean64) / sd64
    g = (0.5 + xhat + 0.5 * torch.randn_like(xhat)).float().to(torch.bfloat16)
    bn.work.scratch.zero_()
    S = _lib.STAT_SLOTS
    bn.work.scratch[: S * 3 * C4].view(S, 3, C4)[0, 1].copy_(g.float().sum(0))  # slab row 1: sum(g)
    bn.weight.grad = torch.zeros(C4, device=DEV)
    bn.bias.grad = torch.zeros(C4, device=DEV)
    bn.work.save.copy_(torch.stack([mean64.float(), (1.0 / sd64).float()]))
    T = gram_T(g.view(N, H, H, C4), h2)
    gram_coef(bn, g.view(N, H, H, C4), T=T, w3=w3, hs=s)
    torch.cuda.synchronize()
    ref = (g.double() * xhat).sum(0)
    e_sgx = float(((bn.weight.grad.double() - ref).abs() / ref.abs()).max())
    print(f"p={p}: x-free sum(g xhat) rel err {e_sgx:.2e}")
    assert float(ref.abs().min()) > 0.1 * M and e_sgx < 1e-3


@pytest.mark.parametrize("C,R", [(64, 5000), (512, 3000), (2048, 700)])
def test_slab_fold_inside_the_pass(C, R):
    """The BN passes fold their statistics slab themselves (SlabFold, bn.hip: the first blocks fold and publish,
    every wave waits on the counter): forward statistics / output and the backward's folded sums and dx equal the
    former separate fold launch's bit for bit."""
    from imagent_amd.ops import _lib
    from imagent_amd.ops.bn import bn_fwd_launch, stats_finalize
    torch.manual_seed(7)
    gamma = torch.rand(C, device=DEV) + 0.5
    beta = torch.randn(C, device=DEV) * 0.1
    x = torch.randn(R, C, device=DEV).to(torch.bfloat16)
    a, b = _work(C), _work(C)
    for rep in range(3):
        a.slab.copy_(torch.randn_like(a.slab) * (rep + 1))
        a.save.copy_(torch.randn_like(a.save))
        b.slab.copy_(a.slab)
        b.scratch.zero_()  # the fold's publish counter (zeroed with the slabs once per step in the model)
        save0 = a.save.clone()
        ya, yb = torch.empty_like(x), torch.empty_like(x)
        b.save.copy_(save0)
        stats_finalize(a, R)
        bn_fwd_launch(x, a.stats, gamma, beta, ya, a.save)
        bn_fwd_launch(x, b.stats, gamma, beta, yb, b.save, fold=b)
        torch.cuda.synchronize()
        assert torch.equal(a.stats, b.stats), rep
        assert torch.equal(ya, yb) and torch.equal(a.save, b.save), rep
    # backward: apply with the fold inside vs the separate launch, on identical slabs
    g = torch.randn(R, C, device=DEV).to(torch.bfloat16)
    k = _lib.kernels()
    res = []
    for fold_in in (0, 1, 1):
        w = _work(C)
        torch.manual_seed(8)
        nb = 32 * 3 * C
        w.scratch[:nb].copy_(torch.randn(nb, device=DEV))
        w.save.copy_(torch.stack([torch.randn(C, device=DEV) * 0.1, torch.rand(C, device=DEV) + 0.5]))
        dx = torch.empty_like(x)
        dg, db = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
        _lib.check(k.imk_bn_bwd_apply(g.data_ptr(), x.data_ptr(), w.save.data_ptr(), gamma.data_ptr(), None, None,
                                      None, w.scratch.data_ptr(), dx.data_ptr(), None, dg.data_ptr(), db.data_ptr(),
                                      None, None, R, C, 0, None, 0, fold_in, _lib.stream_ptr()), "apply")
        torch.cuda.synchronize()
        res.append((dx, w.scratch[nb:nb + 3 * C].clone(), dg, db))
    for r in res[1:]:
        assert torch.equal(r[0], res[0][0]) and torch.equal(r[1], res[0][1])
        assert torch.equal(r[2], res[0][2]) and torch.equal(r[3], res[0][3])
