"""Convolution / linear on the hand-written MFMA implicit-GEMM kernels.

Activations are NHWC bf16 tensors ``[N, H, W, C]``; weights are the fp32
master parameters (torchvision shape ``[Co, Ci, KH, KW]`` stored
channels-last, i.e. ``[Co][KH][KW][Ci]`` in memory) plus two bf16 shadows kept
current by the optimizer step: ``w`` ``[Co][KH][KW][Ci]`` for the forward and
wgrad, ``wt`` ``[Ci][KH][KW][Co]`` for the dgrad.

Reference counterpart: the cuDNN convolutions torchvision's resnet issues
(``/root/reference/imagenet.py:312`` model, fwd ``:123``, bwd ``:128``).
"""

from __future__ import annotations

import contextlib
import ctypes as C
import os
from typing import Optional, Tuple

import torch

from . import _lib, streams
from .grad_sink import notify_ready


def conv_out_size(h: int, k: int, s: int, p: int) -> int:
    return (h + 2 * p - k) // s + 1


def _magic(d: int) -> Tuple[int, int]:
    """Unsigned magic-number division constants: q = (umulhi(n, m) + n) >> s."""
    if d <= 1:
        return 0, 0
    s = (d - 1).bit_length()
    m = ((1 << 32) * ((1 << s) - d)) // d + 1
    return m & 0xFFFFFFFF, s


# IMAGENT_CONV_LOG=<path>: append one JSON line per conv kernel call (op, GEMM shape, flags, kernel
# dispatches it produced, stream) -- joined with a rocprofv3 kernel trace by scripts/conv_roofline.py
_LOG_PATH = os.environ.get("IMAGENT_CONV_LOG")
_log_file = None


def _igemm_call(a, tile: int, st, what: str) -> None:
    k = _lib.kernels()
    if _LOG_PATH is None:
        _lib.check(k.imk_conv_igemm(C.byref(a), tile, st), what)
        return
    n0 = k.imk_conv_launches()
    _lib.check(k.imk_conv_igemm(C.byref(a), tile, st), what)
    _log(dict(op=what, N=a.N, H=a.H, W=a.W, C=a.C, OH=a.OH, OW=a.OW, M=a.M, Nout=a.Nout, taps=a.nth * a.ntw,
              YH=a.YH, YW=a.YW, sY=a.sY, ldy=a.ldy, flags=a.flags, bnb=bool(a.flags & 32), y2=bool(a.bnym),
              x2=bool(a.bnx2), stats=bool(a.stats), xbn=bool(a.xbn), X2=bool(a.X2)),
         k.imk_conv_launches() - n0, st)


def _wgrad_call(a, splits: int, st, what: str) -> None:
    k = _lib.kernels()
    if _LOG_PATH is None:
        _lib.check(k.imk_conv_wgrad(C.byref(a), splits, st), what)
        return
    n0 = k.imk_conv_launches()
    _lib.check(k.imk_conv_wgrad(C.byref(a), splits, st), what)
    _log(dict(op=what, N=a.N, H=a.H, W=a.W, C=a.Ci, Co=a.Co, OH=a.OH, OW=a.OW, M=a.M, KH=a.KH, KW=a.KW,
              stride=a.stride, stem=bool(a.stem), xbn=bool(a.xbn)), k.imk_conv_launches() - n0, st)


def _log(rec, nk: int, st) -> None:
    global _log_file
    import json
    if _log_file is None:
        _log_file = open(_LOG_PATH, "a")
    rec["kernels"] = nk
    rec["stream"] = int(st or 0)
    _log_file.write(json.dumps(rec) + "\n")
    _log_file.flush()


def _base_args(x_ptr, w_ptr, y_ptr, N, H, W, Cin, OH, OW, Nout, ldb, sA) -> _lib.IGemmArgs:
    a = _lib.IGemmArgs()
    a.X, a.Wk, a.Y = x_ptr, w_ptr, y_ptr
    a.bias = None
    a.stats = None
    a.N, a.H, a.W, a.C = N, H, W, Cin
    a.OH, a.OW, a.M = OH, OW, N * OH * OW
    a.Nout, a.ldb, a.sA = Nout, ldb, sA
    return a


# epilogue choice: 0 auto (LDS-staged for fused BN backward, else direct),
# 1 direct register epilogue, 2 LDS-staged coalesced epilogue
_EPI_FLAGS = {0: 0, 1: 128, 2: 64}
# IMAGENT_CONV_STREAM=0: keep short-K 1x1 convs off the streaming kernel
# (conv_stream.hip) -- A/B switch for benchmarks and numerics tests
_NOSTREAM = 2048 if os.environ.get("IMAGENT_CONV_STREAM", "1") == "0" else 0
# IMAGENT_BN_SHIFT=0: forward BN statistics as raw sums (shift 0) -- A/B switch
_SHIFT = os.environ.get("IMAGENT_BN_SHIFT", "1") != "0"


def set_stream(enabled: bool) -> None:
    """Route short-K (C in {64, 128}) 1x1 convs to the streaming kernel or not."""
    global _NOSTREAM
    _NOSTREAM = 0 if enabled else 2048


# Deterministic mode (IMAGENT_DETERMINISTIC=1 or set_deterministic(True); bench / CLI --deterministic): BatchNorm
# statistics without float atomics -- the forward statistics come from a fixed-order pass over the conv output
# (bn.hip bn_stats_det_kernel) instead of the conv epilogue, and the backward reductions from the separate
# reduce pass with a fixed-order fold (the models bind with bnb_fusion off and the unfused stem). Two passes over
# the same data then give bit-identical statistics and activations; the weight gradients' split-K fp32 atomics
# remain (order effects ~1e-7 relative, no feedback within a step).
_DET = os.environ.get("IMAGENT_DETERMINISTIC", "0") == "1"


def deterministic() -> bool:
    return _DET


_DET_LIB = None  # the mode last pushed to the kernel library


def set_deterministic(on: bool) -> None:
    """Switch the deterministic mode (before binding a model: it decides the BN-backward fusion)."""
    global _DET, _DET_LIB
    _DET = bool(on)
    if torch.cuda.is_available():
        _lib.check(_lib.kernels().imk_set_deterministic(1 if _DET else 0), "set deterministic")
        _DET_LIB = _DET


def _det_sync() -> None:
    """The library follows this module's mode (e.g. IMAGENT_DETERMINISTIC=1 in a spawned worker)."""
    if _DET_LIB != _DET:
        set_deterministic(_DET)


def igemm_fwd(x: torch.Tensor, w: torch.Tensor, stride: int, pad: int, KH: int, KW: int,
              stats: Optional[torch.Tensor] = None, bias: Optional[torch.Tensor] = None,
              out_f32: bool = False, relu: bool = False, out: Optional[torch.Tensor] = None,
              tile: int = 0, stem: bool = False, epi: int = 0,
              fp8: Optional[Tuple[torch.Tensor, torch.Tensor]] = None, affine: Optional[torch.Tensor] = None,
              accumulate: bool = False, xbn: Optional[torch.Tensor] = None, res: Optional[torch.Tensor] = None,
              maskout: Optional[torch.Tensor] = None, res_scale: Optional[torch.Tensor] = None,
              q8out=None) -> torch.Tensor:
    """y[N,OH,OW,Co] = conv(x[N,H,W,Ci], w[Co,KH,KW,Ci]) (+bias) (ReLU); optional
    per-channel (sum, sumsq) accumulation into ``stats`` (a [STAT_SLOTS, 2, Co]
    slab), or, given a BatchNorm workspace (``bn.work``), into its slab as
    sums of ``v - shift`` with shift = that BN's previous batch mean
    (``work.save[:Co]``; finalize with :func:`ops.bn.stats_finalize`).

    ``stem``: x has 4 channels and w is ``[Co][KH][32]`` (row = KW taps x 4
    channels, zero padded) - the row-segment gather of the 7x7 stem.
    ``fp8 = (ex, ew)``: x and w are e4m3 bytes (uint8) holding x*2^-ex and
    w*2^-ew, ex/ew device int32 scalars; the block-scaled MFMA restores the
    scales (Ci % 16 == 0).
    ``affine`` [2, Co] fp32 (scale, shift): an inference BatchNorm folded into
    the epilogue (before ``accumulate`` into ``out`` and ``relu``).
    ``xbn`` [2, Ci] fp32 (scale, shift): the operand is relu(x * scale + shift) -- the producing
    BatchNorm's apply + ReLU done on this conv's operand load (1x1, Ci in {64, 128}: the
    streaming kernel; see :func:`ops.bn.bn_scale_shift`).
    ``res`` (like ``out``): added after ``affine`` and before ``relu`` (training: a block's last BatchNorm +
    shortcut + ReLU in the conv's epilogue); ``maskout`` (uint8, numel / 8): also the ReLU mask of the stored
    output as bits; ``res_scale`` (fp32 [Co]): the residual enters as res * res_scale (a downsample block's
    shortcut BatchNorm, its shift folded into ``affine``); ``q8out`` = (y8 uint8 like ``out``, exponent int32[1],
    amax fp32[32]): also the delayed-scaled e4m3 copy of the output. All four: the streaming 1x1 kernel only."""
    N, H, W, Ci = x.shape
    Co = w.shape[0]
    OH, OW = conv_out_size(H, KH, stride, pad), conv_out_size(W, KW, stride, pad)
    if out is None:
        out = torch.empty((N, OH, OW, Co), device=x.device,
                          dtype=torch.float32 if out_f32 else torch.bfloat16)
    if stem:
        assert Ci == 4 and tuple(w.shape) == (Co, KH, 32), (x.shape, w.shape)
    a = _base_args(x.data_ptr(), w.data_ptr(), out.data_ptr(), N, H, W, Ci, OH, OW, Co,
                   KH * 32 if stem else KH * KW * Ci, stride)
    a.nth, a.ntw, a.dh0, a.dhs, a.dw0, a.dws = KH, KW, -pad, 1, -pad, 1
    a.kh0, a.khs, a.kw0, a.kws, a.KW = 0, 1, 0, 1, KW
    a.YH, a.YW, a.sY, a.oy, a.ox, a.ldy = OH, OW, 1, 0, 0, Co
    a.flags = (1 if out_f32 else 0) | (2 if relu else 0) | (4 if stem else 0) | _EPI_FLAGS[epi] | \
        (8 if accumulate else 0) | _NOSTREAM
    if affine is not None:
        assert bias is None and affine.shape == (2, Co) and affine.dtype == torch.float32
        a.flags |= 1024
        a.bias = affine.data_ptr()
    if res is not None:
        assert res.shape == out.shape and res.dtype == torch.bfloat16 and res.is_contiguous()
        a.flags |= 8192
        a.bnx = res.data_ptr()
        if res_scale is not None:
            assert res_scale.dtype == torch.float32 and res_scale.numel() == Co and res_scale.is_contiguous()
            a.bnsave2 = res_scale.data_ptr()
    if q8out is not None:
        y8, e8, a8 = q8out
        assert y8.dtype == torch.uint8 and y8.numel() == out.numel() and e8.dtype == torch.int32
        a.flags |= 32768
        a.Y8, a.y8exp, a.y8amax = y8.data_ptr(), e8.data_ptr(), a8.data_ptr()
    if maskout is not None:
        assert maskout.dtype == torch.uint8 and maskout.numel() * 8 == out.numel() and relu
        a.flags |= 16384
        a.bnym = maskout.data_ptr()
    if fp8 is not None:
        assert x.dtype == torch.uint8 and w.dtype == torch.uint8, (x.dtype, w.dtype)
        a.flags |= 256
        a.xexp, a.wexp = fp8[0].data_ptr(), fp8[1].data_ptr()
    if bias is not None:
        a.bias = bias.data_ptr()
    if xbn is not None:
        assert xbn.shape == (2, Ci) and xbn.dtype == torch.float32 and xbn.is_contiguous()
        a.xbn = xbn.data_ptr()
    det = None
    if stats is not None:
        if hasattr(stats, "slab"):  # a BatchNorm's workspace: shifted sums around its last batch mean
            if _SHIFT:
                a.shift = stats.save.data_ptr()
            stats = stats.slab
        if _DET and not out_f32 and x.is_cuda:  # statistics by the fixed-order pass below
            det, a.shift = (stats, a.shift), None
        else:
            a.stats = stats.data_ptr()
    _igemm_call(a, tile, _lib.stream_ptr(), "conv fwd")
    if det is not None:
        _det_sync()
        k, R = _lib.kernels(), out.numel() // Co
        part = torch.empty(k.imk_bn_stats_det_floats(R, Co), device=out.device, dtype=torch.float32)
        _lib.check(k.imk_bn_stats_det(out.data_ptr(), det[1], det[0].data_ptr(), part.data_ptr(), R, Co,
                                      _lib.stream_ptr()), "bn stats (deterministic)")
    return out


def igemm_dgrad(dy: torch.Tensor, wt: torch.Tensor, in_hw: Tuple[int, int], stride: int, pad: int,
                KH: int, KW: int, out: Optional[torch.Tensor] = None,
                accumulate: bool = False, tile: int = 0, bnb: Optional["BNBwdFuse"] = None,
                epi: int = 0, fp8=None, sparse: bool = False, old_sub2: bool = False) -> torch.Tensor:
    """dx[N,H,W,Ci] (+)= dgrad(dy[N,OH,OW,Co], wt[Ci,KH,KW,Co]).

    Stride 1: one gather-GEMM launch with the taps mirrored.
    Stride s: s*s launches, one per output parity class, each touching only
    the taps that hit it (sub-pixel decomposition: no multiply-by-zero work).
    ``accumulate``: the epilogue adds into ``out`` (fuses a residual-branch
    gradient sum into the store instead of a separate add kernel).
    ``bnb``: ``dx`` is the upstream gradient of that BatchNorm(+add)+ReLU: the
    epilogue stores it ReLU-masked and adds the BN-backward reductions to the
    BN's slab (finish with :func:`ops.bn.bn_apply_backward`).
    ``fp8 = (dy8, exp_dy, wt8, exp_w)``: e5m2 gradient x e4m3 transposed
    weights on the block-scaled MFMA (device int32 exponents).
    ``sparse`` (stride 2, 1x1): write only the computed parity class, no memset
    of the others -- the caller's next dgrad accumulates with ``old_sub2``.
    ``old_sub2`` (with ``accumulate``): ``out`` holds valid values only at even
    (y, x) pixels (a ``sparse`` stride-2 dgrad), zeros elsewhere by definition.
    """
    assert not accumulate or out is not None
    N, OH, OW, Co = dy.shape
    Ci = wt.shape[0]
    H, W = in_hw
    if out is None:
        out = torch.empty((N, H, W, Ci), device=dy.device, dtype=torch.bfloat16)
    k = _lib.kernels()
    st = _lib.stream_ptr()
    S = stride
    if not accumulate and S > 1 and (KH < S or KW < S):
        # some parity classes get no tap (e.g. a strided 1x1): one memset of
        # the output instead of zero-producing GEMM launches for those classes
        # (sparse: no memset either; the consumer knows those pixels are zero)
        if sparse:
            assert S == 2 and KH == 1 and KW == 1 and pad == 0, "sparse: stride-2 1x1 dgrads only"
        else:
            _lib.zero_(out)
        skip_empty = True
    else:
        skip_empty = accumulate
    for ph in range(S):
        for pw in range(S):
            gh = (H - ph + S - 1) // S  # rows of this parity class
            gw = (W - pw + S - 1) // S
            if gh <= 0 or gw <= 0:
                continue
            kh0 = (ph + pad) % S
            kw0 = (pw + pad) % S
            nth = max(0, (KH - kh0 + S - 1) // S)
            ntw = max(0, (KW - kw0 + S - 1) // S)
            if skip_empty and (nth == 0 or ntw == 0):
                if bnb is not None:
                    raise NotImplementedError("fused BN backward needs every parity class computed")
                continue  # no tap reaches this parity class: zero / nothing to add
            if fp8 is None:
                a = _base_args(dy.data_ptr(), wt.data_ptr(), out.data_ptr(), N, OH, OW, Co, gh, gw, Ci,
                               KH * KW * Co, 1)
            else:
                a = _base_args(fp8[0].data_ptr(), fp8[2].data_ptr(), out.data_ptr(), N, OH, OW, Co, gh, gw, Ci,
                               KH * KW * Co, 1)
                a.xexp, a.wexp = fp8[1].data_ptr(), fp8[3].data_ptr()
            a.nth, a.ntw = nth, ntw
            a.dh0, a.dhs = (ph + pad - kh0) // S, -1
            a.dw0, a.dws = (pw + pad - kw0) // S, -1
            a.kh0, a.khs, a.kw0, a.kws, a.KW = kh0, S, kw0, S, KW
            a.YH, a.YW, a.sY, a.oy, a.ox, a.ldy = H, W, S, ph, pw, Ci
            a.flags = (8 if accumulate else 0) | _EPI_FLAGS[epi] | (256 | 512 if fp8 is not None else 0) | _NOSTREAM | \
                (4096 if (accumulate and old_sub2) else 0)
            if bnb is not None:
                bnb.fill(a)
            _igemm_call(a, tile, st, "conv dgrad")
    return out


class BNBwdFuse:
    """The BatchNorm a dgrad's output flows into (IG_BNBWD epilogue).

    x: BN input; y: the ReLU mask of the BN(+add)+ReLU output as bits (uint8, numel / 8, written by the
    forward's ``bn_act_forward(ym=)``; ``ops.bn.relu_mask_bits``), None: mask recomputed from x with
    gamma/beta (plain BN+ReLU); x2/bn2: the downsample BN branch of a fused residual (mode 2)."""

    __slots__ = ("x", "y", "bn", "x2", "bn2")

    def __init__(self, x, bn, y=None, x2=None, bn2=None):
        self.x, self.bn, self.y, self.x2, self.bn2 = x, bn, y, x2, bn2

    def fill(self, a) -> None:
        w = self.bn.work
        a.flags |= 32
        a.stats = w.scratch.data_ptr()
        # x None (with the mask bits): the epilogue never reads x; sum(g xhat) is then formed from g^T h2 by the
        # Gram-form bn3 backward (ops/bn_gram.py gram_coef with T)
        assert self.x is not None or self.y is not None, "BNBwdFuse without x: the mask bits are required"
        a.bnx = _lib.ptr(self.x)
        assert self.y is None or self.y.dtype == torch.uint8, "BNBwdFuse.y: the ReLU mask bits"
        a.bnym = _lib.ptr(self.y)
        a.bnsave = w.save.data_ptr()
        a.bngamma = self.bn.weight.data_ptr()
        a.bnbeta = self.bn.bias.data_ptr()
        a.bnx2 = _lib.ptr(self.x2)
        a.bnsave2 = self.bn2.work.save.data_ptr() if self.x2 is not None else None


def igemm_wgrad(dy: torch.Tensor, x: torch.Tensor, dw: torch.Tensor, stride: int, pad: int, KH: int,
                KW: int, splits: int = 0, stem: bool = False, xbn: Optional[torch.Tensor] = None,
                variant: int = 0) -> None:
    """dw[Co, KH*KW*Ci] (fp32, contiguous rows) += wgrad(dy[N,OH,OW,Co], x[N,H,W,Ci]).
    ``stem``: x has 4 channels, dw is ``[Co][KH][32]`` (see :func:`igemm_fwd`).
    ``xbn``: the X operand is relu(x * xbn[0] + xbn[1]) (1x1 convs; as in :func:`igemm_fwd`).
    ``variant`` (tests / A/B): 0 the default dispatch, -1 the register-staged kernel (-2: the stem's), 1..4 and 6 the
    LDS-DMA v3 kernel's stage shapes (conv_wgrad_v3.h)."""
    a = _wgrad_args(dy, x, dw, stride, pad, KH, KW, stem, xbn)
    if variant:
        _lib.check(_lib.kernels().imk_conv_wgrad_variant(C.byref(a), splits, variant, _lib.stream_ptr()),
                   f"conv wgrad variant {variant}")
        return
    _wgrad_call(a, splits, _lib.stream_ptr(), "conv wgrad")


def stem_wgrad_bnx(g: torch.Tensor, x: torch.Tensor, gp: torch.Tensor, bnx: torch.Tensor, coef: torch.Tensor,
                   stride: int, pad: int, KH: int, KW: int) -> bool:
    """The stem's weight gradient with its BatchNorm's backward apply fused into the operand staging
    (conv_wgrad_stem.h): gp [Co][KH][32] += wgrad(bf16(A g + B bnx + c), x) with coef = (A, B, c) [3][Co].
    False (nothing launched) when the band kernel does not cover the shape."""
    a = _wgrad_args(g, x, gp, stride, pad, KH, KW, True, None)
    r = _lib.kernels().imk_stem_wgrad_bnx(C.byref(a), bnx.data_ptr(), coef.data_ptr(), _lib.stream_ptr())
    if r == -106:
        return False
    _lib.check(r, "stem wgrad (fused BN apply)")
    return True


def _wgrad_args(dy, x, dw, stride, pad, KH, KW, stem, xbn):
    N, H, W, Ci = x.shape
    _, OH, OW, Co = dy.shape
    if stem:
        assert Ci == 4 and dw.numel() == Co * KH * 32
    a = _lib.WgradArgs()
    a.stem = 1 if stem else 0
    a.dY, a.X, a.dW = dy.data_ptr(), x.data_ptr(), dw.data_ptr()
    a.N, a.H, a.W, a.Ci, a.Co = N, H, W, Ci, Co
    a.OH, a.OW, a.M = OH, OW, N * OH * OW
    a.KH, a.KW, a.stride, a.pad = KH, KW, stride, pad
    a.m_per_split = 0
    a.mg_ohw, a.sh_ohw = _magic(OH * OW)
    a.mg_ow, a.sh_ow = _magic(OW)
    if xbn is not None:
        assert xbn.shape == (2, Ci) and xbn.dtype == torch.float32 and xbn.is_contiguous()
        a.xbn = xbn.data_ptr()
    return a


def colsum_into(x2d: torch.Tensor, out: torch.Tensor) -> None:
    R, Cc = x2d.shape
    _lib.check(_lib.kernels().imk_colsum_bf16(x2d.data_ptr(), out.data_ptr(), R, Cc, _lib.stream_ptr()),
               "colsum")


# --------------------------------------------------------------------------
# autograd
# --------------------------------------------------------------------------

class ConvFn(torch.autograd.Function):
    """NHWC bf16 conv whose weight gradient lands directly in the parameter's
    slot of the flat fp32 gradient arena (``weight.grad``), then signals the
    bucketed reducer. ``weight`` is passed only to anchor the node in the
    graph (the stem conv's input needs no grad); autograd never sees dW."""

    @staticmethod
    def forward(ctx, x, weight, mod, stats):
        y = igemm_fwd(x, mod.w_bf16, mod.stride, mod.padding, mod.kh, mod.kw, stats=stats,
                      stem=getattr(mod, "stem", False))
        ctx.mod = mod
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, dy):
        streams.flush_deferred()  # (per-op path / stem conv: nothing may stay queued past here)
        (x,) = ctx.saved_tensors
        mod = ctx.mod
        dy = dy.contiguous()
        dx = None
        if ctx.needs_input_grad[0]:
            dx = igemm_dgrad(dy, mod.wt_bf16, (x.shape[1], x.shape[2]), mod.stride, mod.padding, mod.kh,
                             mod.kw)
        conv_wgrad(mod, dy, x)
        return dx, None, None, None


def conv_wgrad(mod, dy: torch.Tensor, x: torch.Tensor, xbn: Optional[torch.Tensor] = None) -> None:
    """Accumulate a Conv2d module's weight gradient into its arena slot and
    signal the bucketed reducer (on the wgrad side stream when enabled,
    ``ops/streams.py``). ``xbn``: x is a BatchNorm's INPUT whose apply + ReLU
    the kernel does on its operand staging (:func:`igemm_wgrad`)."""
    side = streams.side_stream(dy.device) if dy.is_cuda else None
    if side is None:
        _conv_wgrad(mod, dy, x, xbn)
        return
    streams.wait(side, torch.cuda.current_stream(dy.device))
    with torch.cuda.stream(side):
        _conv_wgrad(mod, dy, x, xbn)
    if xbn is not None:
        streams.protect(dy, x, xbn)
    else:
        streams.protect(dy, x)
    streams.ensure_join_after_backward()


def _conv_wgrad(mod, dy: torch.Tensor, x: torch.Tensor, xbn: Optional[torch.Tensor] = None) -> None:
    gp = getattr(mod, "grad_pad", None)
    if gp is not None:  # stem: [Co][KH][32] row-segment layout (zero between steps) -> master [Co][KH][KW][Ci]
        igemm_wgrad(dy, x, gp, mod.stride, mod.padding, mod.kh, mod.kw, stem=True)
        g = mod.weight.grad  # the arena's [Co][Ci][KH][KW] view of [Co][KH][KW][Ci] storage
        assert tuple(g.shape) == (gp.shape[0], mod.in_channels, mod.kh, mod.kw) and g.permute(0, 2, 3, 1).is_contiguous()
        _lib.check(_lib.kernels().imk_stem_grad_fold(gp.data_ptr(), g.data_ptr(), gp.shape[0], mod.in_channels,
                                                     mod.kh, mod.kw, _lib.stream_ptr()), "stem grad fold")
    else:
        igemm_wgrad(dy, x, mod.weight.grad, mod.stride, mod.padding, mod.kh, mod.kw, xbn=xbn)
    notify_ready(mod.weight)


class LinearFn(torch.autograd.Function):
    """fc layer as a 1x1 conv on a 1x1 image: x [B, Cin] bf16 -> logits fp32 [B, Cout]."""

    @staticmethod
    def forward(ctx, x, weight, mod):
        B, Cin = x.shape
        y = igemm_fwd(x.view(B, 1, 1, Cin), mod.w_bf16.view(mod.out_features, 1, 1, Cin), 1, 0, 1, 1,
                      bias=mod.bias, out_f32=True)
        ctx.mod = mod
        ctx.save_for_backward(x)
        return y.view(B, -1)

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        mod = ctx.mod
        B, Cin = x.shape
        if dy.dtype == torch.float32 and dy.is_cuda:  # (the xent backward's fp32 gradient: own cast kernel)
            dyb = torch.empty(dy.shape, device=dy.device, dtype=torch.bfloat16)
            _lib.check(_lib.kernels().imk_cast_bf16(dy.contiguous().data_ptr(), dyb.data_ptr(), dy.numel(),
                                                    _lib.stream_ptr()), "cast")
            dyb = dyb.view(B, 1, 1, -1)
        else:
            dyb = dy.to(torch.bfloat16).contiguous().view(B, 1, 1, -1)
        if mod.out_features % 8 == 0:
            dx = igemm_dgrad(dyb, mod.wt_bf16.view(Cin, 1, 1, -1), (1, 1), 1, 0, 1, 1).view(B, Cin)
        else:  # the gather GEMM needs 16-B channel chunks; a class count like 100 takes a library GEMM
            dx = (dyb.view(B, -1) @ mod.w_bf16).view(B, Cin)
        if mod.out_features % 8 == 0:
            igemm_wgrad(dyb, x.view(B, 1, 1, Cin), mod.weight.grad, 1, 0, 1, 1)
        else:
            mod.weight.grad.addmm_(dyb.view(B, -1).t().float(), x.float())
        notify_ready(mod.weight)
        if mod.bias is not None:
            colsum_into(dyb.view(B, -1), mod.bias.grad)
            notify_ready(mod.bias)
        return dx, None, None
