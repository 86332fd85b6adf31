"""A bottleneck's last BatchNorm backward without its apply pass (``csrc/kernels/bn_gram.hip``).

For x3 = conv3(h2) (1x1, p -> 4p) and its BatchNorm bn3 (torchvision Bottleneck, the reference's
``models.resnet50``, imagenet.py:312; backward :128) the backward output dx3 = A g + B x3 + c is the
widest activation gradient of the block. Instead of writing it:

* :func:`gram_coef` turns bn3's reductions (accumulated by the producing dgrad's epilogue) into the
  per-channel (A, B, c) and accumulates dgamma / dbeta;
* :func:`gram_dgrad` runs conv3's dgrad as ONE GEMM over the concatenated operand [g | h2] with the
  weights [diag(A) W3 | W3^T diag(B) W3] and the bias c W3, into bn2's fused backward epilogue;
* :func:`gram_wgrad` forms conv3's weight gradient from g^T h2, the centred Gram matrix
  h2^T h2 - s s^T / M and the column sums s of h2 (side stream), then one fix-up kernel.

Every matrix that enters a variance or a mean-subtracted sum is centred before it is contracted with
W3 (``gram_P``, the x-free ``gram_coef``), so a channel whose |mean| >> std keeps its variance
(tests/test_bn_numerics_gpu.py).

h2 (conv3's input, relu(bn2(x2))) has to exist: blocks that take this path keep it materialised
in forward (``ops/block.py``)."""

from __future__ import annotations


import torch

from . import _lib, streams
from .conv import BNBwdFuse, _base_args, _igemm_call, colsum_into, igemm_wgrad
from .grad_sink import notify_ready

# split-K of the skinny Gram GEMMs (T = g^T h2, G = h2^T h2: a [4p][p] / [p][p] output over M ~ 1e5-3e6 pixels):
# one wave of 512 blocks (2 per CU) on the v3 weight-gradient loop -- scripts/gram_bench.py at 1024 img, isolated:
# G 128x128 90 -> 66 us, 256x256 74 -> 52, T 512x128 223 -> 187, 1024x256 186 -> 167 (the default 1024-block
# target pays a second, partial wave).


def _splits(co: int, ci: int) -> int:
    if co % 128 or ci % 128:  # (the register-staged kernel keeps its own choice)
        return 0
    return max(16, 512 // ((co // 128) * (ci // 128)))


def gram_G(h2: torch.Tensor, G: torch.Tensor) -> None:
    """G += h2^T h2 ([p][p] fp32) on the current stream. p = 64 / 128: the weight-gradient loop with h2 staged ONCE
    and read as both operands (imk_gram_sym; for p = 64 over pixel pairs); otherwise the plain weight gradient.
    At 2048 img (scripts/gram_bench.py): p = 64 @56 275 -> 159 us (5.2 TB/s), p = 128 @28 116 -> 105; in-step
    16,830 / 16,912 vs 16,840 / 16,777 img/s (same box, within noise)."""
    p = h2.shape[-1]
    M = h2.numel() // p
    if p in (64, 128) and M % 2 == 0:
        _lib.check(_lib.kernels().imk_gram_sym(h2.data_ptr(), G.data_ptr(), M, p, 512, _lib.stream_ptr()),
                   "gram G")
        return
    igemm_wgrad(h2, h2, G, 1, 0, 1, 1, splits=_splits(p, p))


class GramBN:
    """bn3's backward output dx3 = A g + B x3 + c, kept as (g, coef = [3][4p] (A, B, c)); T = g^T h2 when
    it was formed for the coefficients (``gram_T``)."""

    __slots__ = ("g", "coef", "T")

    def __init__(self, g: torch.Tensor, coef: torch.Tensor, T: torch.Tensor = None):
        self.g, self.coef, self.T = g, coef, T


def gram_T(g: torch.Tensor, h2: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
    """T = g^T h2 [4p][p] fp32 (conv3's weight-gradient GEMM), on the current stream (``out``: zeroed)."""
    C4, p = g.shape[-1], h2.shape[-1]
    T = out if out is not None else torch.zeros((C4, p), device=g.device, dtype=torch.float32)
    igemm_wgrad(g, h2, T, 1, 0, 1, 1, splits=_splits(g.shape[-1], h2.shape[-1]))
    return T


def gram_coef(bn, g: torch.Tensor, T: torch.Tensor = None, w3: torch.Tensor = None,
              hs: torch.Tensor = None) -> GramBN:
    """(A, B, c) of bn3 from its reduction slab; dgamma / dbeta accumulate as the apply pass would.
    ``T`` (= g^T h2), ``w3`` (conv3's bf16 weight [4p][p]) and ``hs`` (colsum(h2)): sum(g xhat) from them instead
    of the slab, centred per element (the producing dgrad ran without x, BNBwdFuse(None, ...): one read of x3
    less)."""
    w = bn.work
    C = bn.weight.shape[0]
    R = g.numel() // C
    coef = torch.empty((3, C), device=g.device, dtype=torch.float32)
    if T is not None:
        p = T.shape[1]
        assert w3.numel() == C * p and w3.dtype == torch.bfloat16 and hs is not None and hs.numel() == p
        _lib.check(_lib.kernels().imk_bn_bwd_coef_T(w.scratch.data_ptr(), T.data_ptr(), w3.data_ptr(),
                                                    hs.data_ptr(), w.save.data_ptr(), bn.weight.data_ptr(),
                                                    bn.weight.grad.data_ptr(), bn.bias.grad.data_ptr(),
                                                    coef.data_ptr(), R, C, p, _lib.stream_ptr()), "bn bwd coef T")
    else:
        _lib.check(_lib.kernels().imk_bn_bwd_coef(w.scratch.data_ptr(), w.save.data_ptr(), bn.weight.data_ptr(),
                                                  bn.weight.grad.data_ptr(), bn.bias.grad.data_ptr(),
                                                  coef.data_ptr(), R, C, _lib.stream_ptr()), "bn bwd coef")
    notify_ready(bn.weight)
    notify_ready(bn.bias)
    return GramBN(g, coef, T)


def gram_P(conv, G: torch.Tensor, s: torch.Tensor, rows: int, out: torch.Tensor = None) -> torch.Tensor:
    """P = W3 (G - s s^T / rows) [4p][p] fp32: conv3's weight times the CENTRED Gram matrix of h2
    (``bn_gram_gemm_kernel<0>``, split-K: it accumulates into ``out``, a zeroed [4p][p] -- the per-step workspace --
    or a fresh zeroed tensor), on the current stream."""
    C4, p = conv.out_channels, conv.in_channels
    P = out if out is not None else torch.zeros((C4, p), device=G.device, dtype=torch.float32)
    _lib.check(_lib.kernels().imk_bn_gram_p(conv.w_bf16.data_ptr(), G.data_ptr(), s.data_ptr(), P.data_ptr(), rows,
                                            C4, p, _lib.stream_ptr()), "bn gram P")
    return P


def gram_dgrad(gb: GramBN, conv, h2: torch.Tensor, bnb: BNBwdFuse, Q: torch.Tensor = None) -> torch.Tensor:
    """dh2 = dx3 W3 without dx3: one v3 GEMM over K = [g (4p) | h2 (p)] with bn2's fused
    backward epilogue (``bnb``; the bias c W3 enters before its ReLU mask). ``Q``: a zeroed [p][p] fp32 accumulator
    for W3^T diag(B) W3 (the per-step workspace) or None."""
    N, H, W, C4 = gb.g.shape
    p = h2.shape[-1]
    wt = conv.wt_bf16  # [p][1][1][4p] = W3^T
    assert tuple(wt.shape) == (p, 1, 1, C4) and conv.kh == 1 and conv.stride == 1
    wcat = torch.empty((p, C4 + p), device=h2.device, dtype=torch.bfloat16)
    bias = torch.empty((p,), device=h2.device, dtype=torch.float32)
    k = _lib.kernels()
    st = _lib.stream_ptr()
    # Q = W3^T diag(B) W3 [p][p] (symmetric), own fp32 kernel (hipBLASLt ran p = 128 as ONE 128 x 128 workgroup:
    # 36 us alone, 200-360 us in the step beside the weight-gradient stream)
    if Q is None:
        Q = torch.zeros((p, p), device=h2.device, dtype=torch.float32)
    _lib.check(k.imk_bn_gram_q(wt.data_ptr(), C4, gb.coef.data_ptr(), Q.data_ptr(), p, C4, st), "gram Q")
    _lib.check(k.imk_bn_gram_dgrad_weights(wt.data_ptr(), C4, gb.coef.data_ptr(), Q.data_ptr(), wcat.data_ptr(),
                                           bias.data_ptr(), p, C4, st), "gram dgrad weights")
    out = torch.empty((N, H, W, p), device=h2.device, dtype=torch.bfloat16)
    a = _base_args(gb.g.data_ptr(), wcat.data_ptr(), out.data_ptr(), N, H, W, C4, H, W, p, C4 + p, 1)
    a.nth, a.ntw, a.dh0, a.dhs, a.dw0, a.dws = 1, 1, 0, 1, 0, 1
    a.kh0, a.khs, a.kw0, a.kws, a.KW = 0, 1, 0, 1, 1
    a.YH, a.YW, a.sY, a.oy, a.ox, a.ldy = H, W, 1, 0, 0, p
    a.flags = 0
    a.X2, a.C2 = h2.data_ptr(), p
    a.bias = bias.data_ptr()
    bnb.fill(a)
    _igemm_call(a, 0, st, "conv dgrad (bn3 gram)")
    return out


def gram_fwd_stats(bn, conv, h2: torch.Tensor, s: torch.Tensor, G: torch.Tensor, add_shift: torch.Tensor = None,
                   P: torch.Tensor = None):
    """bn3's batch statistics without conv3's output (x3 = h2 W3^T): G = h2^T h2 into the zeroed ``G``, P =
    W3 (G - s s^T / M) (centred), then mean = W3 s / M, var = rowsum(P * W3) / M (``bn_gram_fwd_stats_kernel``)
    into ``bn.work.stats`` / ``save``. Returns (aff [2][4p] = (gamma rstd, beta - mean gamma rstd) for conv3's
    epilogue, P; the weight gradient reuses P). ``add_shift`` [4p]: added to the returned shift (a downsample
    block's shortcut-BN shift, folded into bn3's). ``P``: a zeroed [4p][p] accumulator (workspace) or None."""
    C4, p = conv.out_channels, conv.in_channels
    M = h2.numel() // p
    gram_G(h2, G)
    P = gram_P(conv, G, s, M, out=P)
    aff = torch.empty((2, C4), device=h2.device, dtype=torch.float32)
    w = bn.work
    _lib.check(_lib.kernels().imk_bn_gram_fwd_stats(conv.w_bf16.data_ptr(), s.data_ptr(), P.data_ptr(),
                                                    bn.weight.data_ptr(), bn.bias.data_ptr(), w.stats.data_ptr(),
                                                    w.save.data_ptr(), aff.data_ptr(), _lib.ptr(add_shift), M, C4, p,
                                                    float(bn.eps), _lib.stream_ptr()), "bn gram fwd stats")
    return aff, P


def gram_wgrad(conv, gb: GramBN, h2: torch.Tensor, s: torch.Tensor = None, G: torch.Tensor = None,
               P: torch.Tensor = None, bn=None, T_out: torch.Tensor = None, P_out: torch.Tensor = None):
    """conv3.weight.grad += A (g^T h2) + B W3 Gc + (c + B mean) colsum(h2) (Gc = the centred Gram matrix of h2;
    ``bn``: bn3, whose saved batch mean enters), on the wgrad side stream.
    ``s``: colsum(h2) if the forward already accumulated it (``bn_act_forward(colsum=)``); ``G``: a zeroed
    [p][p] fp32 accumulator (the per-step workspace) or None; ``P`` = W3 Gc when the forward already formed it
    (``gram_fwd_stats``): then neither G nor P is recomputed. ``T_out`` / ``P_out``: zeroed accumulators for T / P
    when they are formed here (the per-step workspace), else fresh zeroed tensors.
    Returns the side-stream event after the last read of ``g`` (or None without a side stream):
    the caller's next writer of ``g`` (conv1's accumulating dgrad) waits for it."""
    if bn is None:  # its saved batch mean enters the fix-up, and the side stream protects its workspace
        raise ValueError("gram_wgrad needs bn (the block's bn3)")
    side = streams.side_stream(h2.device) if h2.is_cuda else None
    if side is not None:
        streams.wait(side, torch.cuda.current_stream(h2.device))
    ctx = torch.cuda.stream(side) if side is not None else _Null()
    with ctx:
        C4, p = gb.g.shape[-1], h2.shape[-1]
        if G is None and P is None:
            G = torch.zeros((p, p), device=h2.device, dtype=torch.float32)
        own_s = s is None
        if own_s:
            s = torch.zeros((p,), device=h2.device, dtype=torch.float32)
        ev = None
        T = gb.T
        if T is None:  # (else formed on the main stream for the coefficients: g is not read here)
            T = T_out if T_out is not None else torch.zeros((C4, p), device=h2.device, dtype=torch.float32)
            igemm_wgrad(gb.g, h2, T, 1, 0, 1, 1, splits=_splits(C4, p))
            if side is not None:
                ev = torch.cuda.Event()
                ev.record(side)
                if torch.cuda.is_current_stream_capturing():
                    streams._capture_events.append(ev)  # (waited on later; outlives the capture, streams.wait)
        if P is None:
            gram_G(h2, G)
        if own_s:
            colsum_into(h2.view(-1, p), s)
        if P is None:
            P = gram_P(conv, G, s, h2.numel() // p, out=P_out)
        _lib.check(_lib.kernels().imk_bn_gram_wgrad_fixup(conv.weight.grad.data_ptr(), T.data_ptr(), P.data_ptr(),
                                                          gb.coef.data_ptr(), bn.work.save.data_ptr(), s.data_ptr(),
                                                          C4, p, _lib.stream_ptr()), "gram wgrad fixup")
        notify_ready(conv.weight)
    if side is not None:
        streams.protect(*[t for t in (gb.g, gb.coef, h2, s, T, P, bn.work.save) if t is not None])
        streams.ensure_join_after_backward()
    return ev


class _Null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
