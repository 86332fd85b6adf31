"""BatchNorm(+residual add)(+ReLU) on the fused HIP kernels (NHWC bf16).

Training-mode statistics arrive from the producing conv's epilogue as a
``[STAT_SLOTS, 2, C]`` slab of fp32 partial SHIFTED (sum, sum of squares)
around the previous batch mean (no E[x^2] - mean^2 cancellation when
|mean| >> std), folded by one tiny launch into (mean, variance), so the
forward is one streaming pass. ``save`` receives (mean, invstd) for the
backward and is the next step's shift.

Three forms cover torchvision's blocks (reference model: ``imagenet.py:312``):
  mode 0  y = act(bn(x))                       (conv1/conv2 of a block, stem)
  mode 1  y = act(bn(x) + res)                 (last BN of a block, identity shortcut)
  mode 2  y = act(bn(x) + bn_d(x2))            (last BN + downsample BN, fused)
"""

from __future__ import annotations

import ctypes as C
from typing import Optional, Tuple

import torch

from . import _lib
from .grad_sink import notify_ready


def stats_finalize(work, rows: int) -> None:
    """Fold the conv epilogue's [STAT_SLOTS, 2, C] slab of shifted sums (around
    ``work.save[:C]``, the previous batch mean) over ``rows`` values per
    channel into ``work.stats`` [2, C] = (batch mean, biased variance)."""
    from .conv import _SHIFT  # IMAGENT_BN_SHIFT=0: the epilogues summed raw values (shift 0)
    S, _, C = work.slab.shape
    _lib.check(_lib.kernels().imk_bn_stats_finalize(work.slab.data_ptr(), work.save.data_ptr() if _SHIFT else None,
                                                    work.stats.data_ptr(), S, C, rows, _lib.stream_ptr()),
               "bn stats finalize")


def bn_scale_shift(x: torch.Tensor, bn) -> torch.Tensor:
    """Training-mode BatchNorm whose apply + ReLU runs on the consumer conv's operand load
    (``igemm_fwd(xbn=)`` / ``conv_wgrad(xbn=)``): finalize the conv epilogue's statistics of ``x``
    and return ss [2, C] = (gamma * rstd, beta - mean * gamma * rstd); ``bn.work.save`` gets
    (mean, rstd) for the backward and ``bn.work.stats`` (mean, var) for the running statistics,
    exactly as :func:`bn_act_forward` leaves them. One launch; the BN output is never written."""
    from .conv import _SHIFT
    w = bn.work
    S, _, C = w.slab.shape
    R = x.numel() // C
    ss = torch.empty((2, C), device=x.device, dtype=torch.float32)
    _lib.check(_lib.kernels().imk_bn_finalize_affine(w.slab.data_ptr(), w.save.data_ptr(), w.stats.data_ptr(),
                                                     bn.weight.data_ptr(), bn.bias.data_ptr(), ss.data_ptr(), S, C,
                                                     R, bn.eps, 1 if _SHIFT else 0, _lib.stream_ptr()),
               "bn finalize + affine")
    return ss


def bn_fwd_launch(x, stats, gamma, beta, y, save, *, x2=None, stats2=None, gamma2=None, beta2=None,
                  save2=None, mode=0, relu=True, eps=1e-5, eval_mode=False, q8=None, ym=None, colsum=None,
                  fold=None):
    """``q8 = (y8 uint8, exp int32[1], amax f32[1])``: also write the e4m3 copy of y.
    ``ym`` (uint8, numel / 8; modes 1 / 2 with ReLU): also write the mask y > 0 as bits.
    ``colsum`` (fp32 [C], zeroed; mode 0): also accumulate the column sums of the stored y.
    ``fold`` (mode 0, training): the BN's ``work``: the pass folds ``work.slab`` into ``stats`` itself (the
    former :func:`stats_finalize` launch; its counter in ``work.scratch``'s last row)."""
    C = x.shape[-1]
    R = x.numel() // C
    y8, e8, a8 = q8 if q8 is not None else (None, None, None)
    fslab = fshift = fcnt = None
    fS = 0
    if fold is not None:
        from .conv import _SHIFT
        fslab, fS = fold.slab.data_ptr(), fold.slab.shape[0]
        fshift = fold.save.data_ptr() if _SHIFT else None
        fcnt = fold.scratch.data_ptr() + 4 * (fold.scratch.numel() - C + 1)  # word 1 of the last row
    _lib.check(_lib.kernels().imk_bn_fwd(
        x.data_ptr(), stats.data_ptr(), gamma.data_ptr(), beta.data_ptr(), _lib.ptr(x2),
        _lib.ptr(stats2), _lib.ptr(gamma2), _lib.ptr(beta2), y.data_ptr(), _lib.ptr(save),
        _lib.ptr(save2), R, C, mode, 1 if relu else 0, eps, 1 if eval_mode else 0,
        _lib.ptr(y8), _lib.ptr(e8), _lib.ptr(a8), _lib.ptr(ym), _lib.ptr(colsum), fslab, fshift, fcnt, fS,
        _lib.stream_ptr()), "bn fwd")


def relu_mask_bits(y: torch.Tensor) -> torch.Tensor:
    """The bit mask ``bn_fwd(ym=)`` writes, from a bf16 tensor (tests / reference): byte e // 8 of
    the flat NHWC element index e, bit e % 8 = (y > 0)."""
    b = (y.reshape(-1, 8) > 0).to(torch.int32)
    w = torch.tensor([1 << i for i in range(8)], dtype=torch.int32, device=y.device)
    return (b * w).sum(1).to(torch.uint8)


def bn_act_forward(x: torch.Tensor, x2: Optional[torch.Tensor], bn, bn2, mode: int, relu: bool,
                   q8=None, ym: Optional[torch.Tensor] = None, colsum: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Training-mode forward (no autograd): statistics from ``bn.work.slab``;
    ``q8`` / ``ym`` as in :func:`bn_fwd_launch`."""
    y = torch.empty_like(x)
    w, w2 = bn.work, (bn2.work if bn2 is not None else None)
    R = x.numel() // x.shape[-1]
    fold = w if (mode == 0 and w.scratch is not None) else None  # mode 0: the apply pass folds its own slab
    if fold is None:
        stats_finalize(w, R)
    if w2 is not None:
        stats_finalize(w2, R)
    bn_fwd_launch(x, w.stats, bn.weight, bn.bias, y, w.save, x2=x2, fold=fold,
                  stats2=w2.stats if w2 is not None else None,
                  gamma2=bn2.weight if bn2 is not None else None,
                  beta2=bn2.bias if bn2 is not None else None,
                  save2=w2.save if w2 is not None else None, mode=mode, relu=relu, eps=bn.eps, q8=q8, ym=ym,
                  colsum=colsum)
    return y


def bn_act_backward(dy: torch.Tensor, x: torch.Tensor, x2: Optional[torch.Tensor], y: Optional[torch.Tensor],
                    bn, bn2, mode: int, relu: bool,
                    dres: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """Returns (dx, dres | dx2). dgamma/dbeta land in the gradient arena and the
    reducer is notified. Mode 0 + ReLU recomputes the mask from x (y unused)."""
    w = bn.work
    C = x.shape[-1]
    R = x.numel() // C
    dx = torch.empty_like(x)
    if mode == 1 and dres is None:
        dres = torch.empty_like(x)
    dx2 = torch.empty_like(x2) if mode == 2 else None
    rmode = (2 if mode == 0 else 1) if relu else 0
    _lib.check(_lib.kernels().imk_bn_bwd(
        dy.data_ptr(), y.data_ptr() if rmode == 1 else 0, x.data_ptr(), w.save.data_ptr(),
        bn.weight.data_ptr(), bn.bias.data_ptr(), _lib.ptr(x2) if mode == 2 else 0,
        bn2.work.save.data_ptr() if mode == 2 else 0,
        bn2.weight.data_ptr() if mode == 2 else 0, w.scratch.data_ptr(), dx.data_ptr(),
        _lib.ptr(dres) if mode == 1 else 0, _lib.ptr(dx2), bn.weight.grad.data_ptr(),
        bn.bias.grad.data_ptr(), bn2.weight.grad.data_ptr() if mode == 2 else 0,
        bn2.bias.grad.data_ptr() if mode == 2 else 0,
        R, C, mode, rmode, _lib.stream_ptr()), "bn bwd")
    notify_ready(bn.weight)
    notify_ready(bn.bias)
    if mode == 2:
        notify_ready(bn2.weight)
        notify_ready(bn2.bias)
    return dx, (dres if mode == 1 else dx2)


def bn_apply_backward(g: torch.Tensor, x: torch.Tensor, x2: Optional[torch.Tensor], bn, bn2,
                      mode: int, g8=None, slab_of=None, sgx_row: int = 0) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """Backward of act(bn(x) [+ res | + bn2(x2)]) for a gradient ``g`` that its
    producing dgrad already ReLU-masked and reduced into ``bn.work.scratch``
    (``ops.conv.BNBwdFuse``): one streaming apply pass that folds the slab itself (``SlabFold``, bn.hip).
    Returns (dx, dx2 | None); for mode 1 the residual-branch gradient is g.
    ``g8 = ((q, exp, amax) | None, (q2, exp2, amax2) | None)``: also write e5m2
    copies of dx / dx2 for the fp8 dgrad (``Fp8State``).
    ``slab_of`` / ``sgx_row`` (modes 0 / 1): the reductions sit in another BN's slab, sum(g xhat) in its row
    ``sgx_row`` (a Gram-form bn3 whose dgrad epilogue also reduced the downsample BN: ops/block.py)."""
    w = bn.work
    scratch = (slab_of if slab_of is not None else bn).work.scratch
    C = x.shape[-1]
    R = x.numel() // C
    dx = torch.empty_like(x)
    dx2 = torch.empty_like(x2) if mode == 2 else None
    _lib.check(_lib.kernels().imk_bn_bwd_apply(
        g.data_ptr(), x.data_ptr(), w.save.data_ptr(), bn.weight.data_ptr(), _lib.ptr(x2),
        bn2.work.save.data_ptr() if mode == 2 else 0, bn2.weight.data_ptr() if mode == 2 else 0,
        scratch.data_ptr(), dx.data_ptr(), _lib.ptr(dx2), bn.weight.grad.data_ptr(),
        bn.bias.grad.data_ptr(), bn2.weight.grad.data_ptr() if mode == 2 else 0,
        bn2.bias.grad.data_ptr() if mode == 2 else 0, R, C, mode, _g8desc(g8), sgx_row, 1, _lib.stream_ptr()),
        "bn bwd apply")
    notify_ready(bn.weight)
    notify_ready(bn.bias)
    if mode == 2:
        notify_ready(bn2.weight)
        notify_ready(bn2.bias)
    return dx, dx2


def _g8desc(g8):
    if g8 is None or (g8[0] is None and g8[1] is None):
        return None
    a, b = g8
    arr = (C.c_void_p * 6)(_lib.ptr(a[0]) if a else 0, _lib.ptr(b[0]) if b else 0,
                           _lib.ptr(a[1]) if a else 0, _lib.ptr(b[1]) if b else 0,
                           _lib.ptr(a[2]) if a else 0, _lib.ptr(b[2]) if b else 0)
    _g8desc.keep = arr  # alive until the (synchronous) launch call returns
    return C.cast(arr, C.c_void_p)


class BNActFn(torch.autograd.Function):
    """y = act(bn(x) [+ res | + bn2(x2)]) as an autograd node (stem, tests)."""

    @staticmethod
    def forward(ctx, x, x2, bn, bn2, mode, relu):
        y = bn_act_forward(x, x2, bn, bn2, mode, relu)
        ctx.bn, ctx.bn2, ctx.mode, ctx.relu = bn, bn2, mode, relu
        ctx.save_for_backward(x, x2 if mode == 2 else None, y if mode != 0 else None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, x2, y = ctx.saved_tensors
        dx, dsecond = bn_act_backward(dy.contiguous(), x, x2, y, ctx.bn, ctx.bn2, ctx.mode, ctx.relu)
        return dx, dsecond, None, None, None, None


def bn_eval(x, bn, relu, x2=None, bn2=None, mode=0):
    """Inference BN (running statistics), same fusions, no autograd."""
    y = torch.empty_like(x)
    rs = torch.stack([bn.running_mean, bn.running_var])
    rs2 = torch.stack([bn2.running_mean, bn2.running_var]) if bn2 is not None else None
    bn_fwd_launch(x, rs, bn.weight, bn.bias, y, None, x2=x2, stats2=rs2,
                  gamma2=bn2.weight if bn2 is not None else None,
                  beta2=bn2.bias if bn2 is not None else None, mode=mode, relu=relu, eps=bn.eps,
                  eval_mode=True)
    return y


def running_update(desc_tensor: torch.Tensor, n: int) -> None:
    """One launch updates running_mean/var and num_batches_tracked of every BN."""
    _lib.check(_lib.kernels().imk_bn_running_update(desc_tensor.data_ptr(), n, _lib.stream_ptr()),
               "bn running update")
