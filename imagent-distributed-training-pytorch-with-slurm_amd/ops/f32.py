"""fp32 ops on the hand-written kernels of ``csrc/kernels/f32.hip`` -- the reference's own precision.

The reference trains in fp32 (no AMP; ``/root/reference/imagenet.py:312`` model, fwd ``:123``,
loss ``:124``, bwd ``:128``). These autograd Functions run ResNet training at fp32 accuracy on
the framework's own kernels: NHWC fp32 activations, convolutions on the exact-f32 MFMA, weight
gradients written straight into the parameters' slots of the flat gradient arena (then the
bucketed reducer is notified, as on the bf16 path), BatchNorm with deterministic fixed-order
statistics. Every op is checked against the PyTorch fp32 op at <= 1e-4 relative
(``tests/test_f32_gpu.py``).
"""

from __future__ import annotations

import ctypes as C
from typing import Optional, Sequence, Tuple

import torch

from . import _lib, streams
from .conv import _base_args, conv_out_size
from .grad_sink import notify_ready


def _k():
    return _lib.kernels()


# ------------------------------------------------------------------ convolution
def set_split(on: bool) -> None:
    """fp32 conv (forward / dgrad / wgrad) arithmetic: False (default) exact f32 MFMA; True the 3 x bf16 split
    (hi*hi + hi*lo + lo*hi on the bf16 MFMA, ~2^-16 relative per product, within 1e-4 of fp32 convs;
    f32.hip igemm_f32s_kernel / wgrad_f32s_kernel; bench.py --fp32-split)."""
    _lib.check(_k().imk_set_f32_split(1 if on else 0), "set f32 split")


def conv_f32(x: torch.Tensor, wk: torch.Tensor, stride: int, pad: int, KH: int, KW: int,
             bias: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
             accumulate: bool = False, stats: Optional[torch.Tensor] = None,
             shift: Optional[torch.Tensor] = None):
    """y[N,OH,OW,Co] (+)= conv(x[N,H,W,Ci], wk[Co][KH][KW][Ci]) (+ bias), fp32 NHWC.
    ``stats`` ([STAT_SLOTS, 2, Co] fp32, zeroed; ``shift`` [Co]): also accumulate the output's BatchNorm
    statistics as sums shifted by ``shift`` in the conv epilogue (the v3 split kernel); then returns
    (y, fused) -- fused False when the kernel taking this shape has no statistics epilogue."""
    N, H, W, Ci = x.shape
    Co = wk.shape[0]
    assert x.dtype == torch.float32 and wk.dtype == torch.float32 and x.is_contiguous() and wk.is_contiguous()
    OH, OW = conv_out_size(H, KH, stride, pad), conv_out_size(W, KW, stride, pad)
    if out is None:
        out = torch.empty((N, OH, OW, Co), device=x.device, dtype=torch.float32)
    a = _base_args(x.data_ptr(), wk.data_ptr(), out.data_ptr(), N, H, W, Ci, OH, OW, Co, KH * KW * Ci, stride)
    a.nth, a.ntw, a.dh0, a.dhs, a.dw0, a.dws = KH, KW, -pad, 1, -pad, 1
    a.kh0, a.khs, a.kw0, a.kws, a.KW = 0, 1, 0, 1, KW
    a.YH, a.YW, a.sY, a.oy, a.ox, a.ldy = OH, OW, 1, 0, 0, Co
    a.flags = 1 | (8 if accumulate else 0)
    if bias is not None:
        a.bias = bias.data_ptr()
    if stats is not None:
        a.stats = stats.data_ptr()
        a.shift = _lib.ptr(shift)
    rc = _k().imk_conv_f32(C.byref(a), _lib.stream_ptr())
    if rc != 2:
        _lib.check(rc, "conv f32")
    if stats is not None:
        return out, rc == 0
    return out


def dgrad_f32(dy: torch.Tensor, wt: torch.Tensor, in_hw: Tuple[int, int], stride: int, pad: int, KH: int,
              KW: int, out: Optional[torch.Tensor] = None, accumulate: bool = False, bnb=None):
    """dx[N,H,W,Ci] (+)= dgrad(dy[N,OH,OW,Co], wt[Ci][KH][KW][Co]); strided convs as one launch per output
    parity class touching only the taps that reach it (the bf16 path's sub-pixel decomposition,
    ops/conv.py igemm_dgrad). ``accumulate``: added to ``out`` in the epilogue (the residual gradient).
    ``bnb = (x, save, bn)``: dx is the upstream gradient of that ReLU'd BatchNorm (input x, save = (mean,
    rstd)): the epilogue stores it masked and sums the BN-backward reductions into ``bn._f32_slab``; returns
    (dx, fused) -- fused False when the kernel taking the shape has no such epilogue (dx then unmasked)."""
    N, OH, OW, Co = dy.shape
    Ci = wt.shape[0]
    H, W = in_hw
    if out is None:
        out = torch.empty((N, H, W, Ci), device=dy.device, dtype=torch.float32)
        accumulate = False
    S = stride
    if S > 1 and (KH < S or KW < S) and not accumulate:
        out.zero_()  # parity classes no tap reaches stay 0
    fused = bnb is not None
    slab = _stats_slab(bnb[2]) if bnb is not None else None
    for ph in range(S):
        for pw in range(S):
            gh, gw = (H - ph + S - 1) // S, (W - pw + S - 1) // S
            if gh <= 0 or gw <= 0:
                continue
            kh0, kw0 = (ph + pad) % S, (pw + pad) % S
            nth, ntw = max(0, (KH - kh0 + S - 1) // S), max(0, (KW - kw0 + S - 1) // S)
            if nth == 0 or ntw == 0:
                continue
            a = _base_args(dy.data_ptr(), wt.data_ptr(), out.data_ptr(), N, OH, OW, Co, gh, gw, Ci, KH * KW * Co, 1)
            a.nth, a.ntw = nth, ntw
            a.dh0, a.dhs = (ph + pad - kh0) // S, -1
            a.dw0, a.dws = (pw + pad - kw0) // S, -1
            a.kh0, a.khs, a.kw0, a.kws, a.KW = kh0, S, kw0, S, KW
            a.YH, a.YW, a.sY, a.oy, a.ox, a.ldy = H, W, S, ph, pw, Ci
            a.flags = 1 | (8 if accumulate else 0)
            if bnb is not None:
                x, save, bn = bnb
                a.flags |= 32  # IG_BNBWD
                a.bnx, a.bnsave, a.stats = x.data_ptr(), save.data_ptr(), slab.data_ptr()
                a.bngamma, a.bnbeta = bn.weight.data_ptr(), bn.bias.data_ptr()
            rc = _k().imk_conv_f32(C.byref(a), _lib.stream_ptr())
            if rc != 2:
                _lib.check(rc, "conv dgrad f32")
            fused = fused and rc == 0
    if bnb is not None:
        return out, fused
    return out


def wgrad_f32(dy: torch.Tensor, x: torch.Tensor, dw: torch.Tensor, stride: int, pad: int, KH: int,
              KW: int) -> None:
    """dw[Co][KH][KW][Ci] (fp32, contiguous) += wgrad(dy[N,OH,OW,Co], x[N,H,W,Ci])."""
    N, H, W, Ci = x.shape
    _, OH, OW, Co = dy.shape
    assert dw.dtype == torch.float32 and dw.numel() == Co * KH * KW * Ci
    _lib.check(_k().imk_wgrad_f32(dy.data_ptr(), x.data_ptr(), dw.data_ptr(), N, H, W, Ci, Co, OH, OW, KH, KW,
                                  stride, pad, _lib.stream_ptr()), "wgrad f32")


def _weight_nhwc(mod, cpad: int = 0) -> torch.Tensor:
    """The fp32 master weight as [Co][KH][KW][Ci] (its channels-last memory; the stem padded to
    ``cpad`` input channels)."""
    w = mod.weight.detach().permute(0, 2, 3, 1)
    if cpad and cpad != w.shape[-1]:
        wp = torch.zeros(w.shape[:3] + (cpad,), device=w.device, dtype=torch.float32)
        wp[..., : w.shape[-1]] = w
        return wp
    return w.contiguous()


def _stats_slab(bn) -> torch.Tensor:
    """The per-BatchNorm [STAT_SLOTS, 2, C] slab the producing conv's epilogue fills (zeroed here)."""
    s = getattr(bn, "_f32_slab", None)
    if s is None or s.device != bn.weight.device:
        s = torch.zeros((_lib.STAT_SLOTS, 2, bn.num_features), device=bn.weight.device, dtype=torch.float32)
        bn._f32_slab = s
    else:
        s.zero_()
    return s


class ConvF32Fn(torch.autograd.Function):
    """NHWC fp32 conv; the weight gradient lands in the parameter's arena slot (``weight.grad``) and
    the bucketed reducer is notified, as ``ops.conv.ConvFn`` does on the bf16 path. The dgrad (critical
    path) is issued first; the weight gradient runs on the side stream (``ops/streams.py``) beside the
    next layers' backward when the overlap is on."""

    @staticmethod
    def forward(ctx, x, weight, mod, bn=None):
        """``bn``: the training BatchNorm that consumes y -- its batch statistics come out of this conv's
        epilogue when the kernel has one (``bn._f32_stats_ready``; :func:`bn_train_f32` folds them)."""
        wk = _weight_nhwc(mod, x.shape[-1])
        if bn is not None:
            y, fused = conv_f32(x, wk, mod.stride, mod.padding, mod.kh, mod.kw, stats=_stats_slab(bn),
                                shift=bn.running_mean)
            bn._f32_stats_ready = fused
        else:
            y = conv_f32(x, wk, mod.stride, mod.padding, mod.kh, mod.kw)
        ctx.mod = mod
        ctx.save_for_backward(x, wk)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wk = ctx.saved_tensors
        mod = ctx.mod
        dy = dy.contiguous()
        dx = None
        if ctx.needs_input_grad[0]:
            wt = wk.permute(3, 1, 2, 0).contiguous()  # [Ci][KH][KW][Co]
            dx = dgrad_f32(dy, wt, (x.shape[1], x.shape[2]), mod.stride, mod.padding, mod.kh, mod.kw)
        g = mod.weight.grad.permute(0, 2, 3, 1)  # arena view, [Co][KH][KW][Ci] memory
        side = streams.side_stream(dy.device) if dy.is_cuda else None
        if side is not None:
            streams.wait(side, torch.cuda.current_stream(dy.device))
        with torch.cuda.stream(side) if side is not None else _nullctx():
            if x.shape[-1] != mod.in_channels:  # stem: 4-channel input, 3-channel weight
                gp = torch.zeros_like(wk)
                wgrad_f32(dy, x, gp, mod.stride, mod.padding, mod.kh, mod.kw)
                g.add_(gp[..., : mod.in_channels])
            else:
                assert g.is_contiguous()
                wgrad_f32(dy, x, g, mod.stride, mod.padding, mod.kh, mod.kw)
            notify_ready(mod.weight)
        if side is not None:
            streams.protect(dy, x)
            streams.ensure_join_after_backward()
        return dx, None, None, None


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


class LinearF32Fn(torch.autograd.Function):
    """fc: x [B, Cin] fp32 -> logits [B, Cout] fp32 (a 1x1 conv on a 1x1 image + bias)."""

    @staticmethod
    def forward(ctx, x, weight, bias, mod):
        B, Cin = x.shape
        w = mod.weight.detach()
        y = conv_f32(x.view(B, 1, 1, Cin), w.view(w.shape[0], 1, 1, Cin), 1, 0, 1, 1, bias=mod.bias.detach())
        ctx.mod = mod
        ctx.save_for_backward(x)
        return y.view(B, -1)

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        mod = ctx.mod
        B, Cin = x.shape
        Cout = dy.shape[1]
        dy = dy.contiguous().float()
        wt = mod.weight.detach().t().contiguous()  # [Cin][Cout]
        dx = conv_f32(dy.view(B, 1, 1, Cout), wt.view(Cin, 1, 1, Cout), 1, 0, 1, 1).view(B, Cin)
        wgrad_f32(dy.view(B, 1, 1, Cout), x.view(B, 1, 1, Cin), mod.weight.grad, 1, 0, 1, 1)
        _lib.check(_k().imk_colsum_f32(dy.data_ptr(), mod.bias.grad.data_ptr(), B, Cout, _lib.stream_ptr()),
                   "colsum f32")
        notify_ready(mod.weight)
        notify_ready(mod.bias)
        return dx, None, None, None


# ------------------------------------------------------------------ BatchNorm
class F32Workspace:
    """Scratch shared by every fp32 BatchNorm of a model (one stream, kernels run in order)."""

    def __init__(self, device, cmax: int):
        self.slab = torch.empty(_k().imk_bn_slab_floats_f32(cmax), device=device, dtype=torch.float32)
        self.red = torch.empty(2 * cmax, device=device, dtype=torch.float32)


def bn_train_f32(x: torch.Tensor, bn, ws: F32Workspace, res: Optional[torch.Tensor], relu: bool):
    """Training BN (+ residual) (+ ReLU): batch statistics (deterministic fold), running stats
    updated; returns (y, save [2, C] = mean, rstd)."""
    C = x.shape[-1]
    R = x.numel() // C
    save = torch.empty(2, C, device=x.device, dtype=torch.float32)
    if getattr(bn, "_f32_stats_ready", False):  # the producing conv's epilogue summed them (ConvF32Fn bn=)
        bn._f32_stats_ready = False
        _lib.check(_k().imk_bn_fold_slab_f32(bn._f32_slab.data_ptr(), bn.running_mean.data_ptr(), save.data_ptr(),
                                             bn.running_mean.data_ptr(), bn.running_var.data_ptr(), R, C,
                                             float(bn.eps), float(bn.momentum), _lib.stream_ptr()), "bn fold f32")
    else:
        # the running mean is the shift of the (shifted) sums: close to the batch mean
        _lib.check(_k().imk_bn_stats_f32(x.data_ptr(), bn.running_mean.data_ptr(), ws.slab.data_ptr(),
                                         save.data_ptr(), bn.running_mean.data_ptr(), bn.running_var.data_ptr(), R,
                                         C, float(bn.eps), float(bn.momentum), _lib.stream_ptr()), "bn stats f32")
    bn.num_batches_tracked.add_(1)
    y = torch.empty_like(x)
    _lib.check(_k().imk_bn_apply_f32(x.data_ptr(), save.data_ptr(), bn.weight.data_ptr(), bn.bias.data_ptr(),
                                     _lib.ptr(res), y.data_ptr(), R, C, int(relu), _lib.stream_ptr()),
               "bn apply f32")
    return y, save


def bn_eval_f32(x: torch.Tensor, bn, res: Optional[torch.Tensor], relu: bool) -> torch.Tensor:
    C = x.shape[-1]
    save = torch.stack([bn.running_mean, torch.rsqrt(bn.running_var + bn.eps)]).float().contiguous()
    y = torch.empty_like(x)
    _lib.check(_k().imk_bn_apply_f32(x.data_ptr(), save.data_ptr(), bn.weight.data_ptr(), bn.bias.data_ptr(),
                                     _lib.ptr(res), y.data_ptr(), x.numel() // C, C, int(relu),
                                     _lib.stream_ptr()), "bn eval f32")
    return y


class BNF32Fn(torch.autograd.Function):
    """y = [ReLU](BN(x) [+ res]); backward: g' = g * (y > 0) -> BN backward (dgamma / dbeta into the
    arena + reducer notification), dres = g'."""

    @staticmethod
    def forward(ctx, x, res, bn, relu, ws):
        y, save = bn_train_f32(x, bn, ws, res, relu)
        ctx.bn, ctx.relu, ctx.ws, ctx.has_res = bn, relu, ws, res is not None
        ctx.save_for_backward(x, y if relu else None, save)
        return y

    @staticmethod
    def backward(ctx, g):
        x, y, save = ctx.saved_tensors
        bn = ctx.bn
        C = x.shape[-1]
        R = x.numel() // C
        g = g.contiguous()
        dx = torch.empty_like(x)
        dres = torch.empty_like(x) if ctx.has_res else None
        _lib.check(_k().imk_bn_bwd_f32(g.data_ptr(), _lib.ptr(y), x.data_ptr(), save.data_ptr(),
                                       bn.weight.data_ptr(), ctx.ws.slab.data_ptr(), ctx.ws.red.data_ptr(),
                                       bn.weight.grad.data_ptr(), bn.bias.grad.data_ptr(), dx.data_ptr(),
                                       _lib.ptr(dres), R, C, _lib.stream_ptr()), "bn bwd f32")
        notify_ready(bn.weight)
        notify_ready(bn.bias)
        return dx, dres, None, None, None


# ------------------------------------------------------------------ residual block
def _bn_bwd(g, y, x, save, bn, ws, want_dres: bool):
    """BN(+ReLU from ``y``) backward of ``g``: (dx, g' = masked g | None); dgamma / dbeta into the arena."""
    C = x.shape[-1]
    R = x.numel() // C
    dx = torch.empty_like(x)
    dres = torch.empty_like(x) if want_dres else None
    _lib.check(_k().imk_bn_bwd_f32(g.data_ptr(), _lib.ptr(y), x.data_ptr(), save.data_ptr(), bn.weight.data_ptr(),
                                   ws.slab.data_ptr(), ws.red.data_ptr(), bn.weight.grad.data_ptr(),
                                   bn.bias.grad.data_ptr(), dx.data_ptr(), _lib.ptr(dres), R, C, _lib.stream_ptr()),
               "bn bwd f32")
    notify_ready(bn.weight)
    notify_ready(bn.bias)
    return dx, dres


def _bn_bwd_slab(g, x, save, bn, ws):
    """BN backward of a gradient the producing dgrad already masked and reduced (dgrad_f32 ``bnb``)."""
    C = x.shape[-1]
    R = x.numel() // C
    dx = torch.empty_like(x)
    _lib.check(_k().imk_bn_bwd_slab_f32(g.data_ptr(), x.data_ptr(), save.data_ptr(), bn.weight.data_ptr(),
                                        bn._f32_slab.data_ptr(), ws.red.data_ptr(), bn.weight.grad.data_ptr(),
                                        bn.bias.grad.data_ptr(), dx.data_ptr(), R, C, _lib.stream_ptr()),
               "bn bwd slab f32")
    notify_ready(bn.weight)
    notify_ready(bn.bias)
    return dx


def _conv_bn_stats(x, conv, bn, fuse: bool):
    """conv_f32 whose epilogue also sums ``bn``'s training statistics when ``fuse`` (bn_train_f32 folds them)."""
    wk = _weight_nhwc(conv, x.shape[-1])
    if not fuse:
        return conv_f32(x, wk, conv.stride, conv.padding, conv.kh, conv.kw)
    y, fused = conv_f32(x, wk, conv.stride, conv.padding, conv.kh, conv.kw, stats=_stats_slab(bn),
                        shift=bn.running_mean)
    bn._f32_stats_ready = fused
    return y


def _wgrad_side(mod, dy, x) -> None:
    """The weight gradient into the arena on the side stream (beside the rest of the backward)."""
    side = streams.side_stream(dy.device) if dy.is_cuda else None
    if side is not None:
        streams.wait(side, torch.cuda.current_stream(dy.device))
    with torch.cuda.stream(side) if side is not None else _nullctx():
        g = mod.weight.grad.permute(0, 2, 3, 1)
        assert g.is_contiguous()
        wgrad_f32(dy, x, g, mod.stride, mod.padding, mod.kh, mod.kw)
        notify_ready(mod.weight)
    if side is not None:
        streams.protect(dy, x)
        streams.ensure_join_after_backward()


def _dgrad(mod, dy, x_shape, out=None, accumulate=False, bnb=None):
    wt = _weight_nhwc(mod).permute(3, 1, 2, 0).contiguous()  # [Ci][KH][KW][Co]
    return dgrad_f32(dy, wt, (x_shape[1], x_shape[2]), mod.stride, mod.padding, mod.kh, mod.kw, out=out,
                     accumulate=accumulate, bnb=bnb)


class BlockF32Fn(torch.autograd.Function):
    """One torchvision residual block (BasicBlock / Bottleneck, with or without downsample) on the fp32
    kernels as ONE autograd node, as the bf16 path's ``ops.block`` does: forward convs with the BatchNorm
    statistics in their epilogues (not in deterministic mode), BN(+residual)(+ReLU) passes; backward
    hand-scheduled: the block-input gradient starts as the residual branch's masked gradient (or the
    downsample dgrad) and conv1's dgrad ACCUMULATES into it in its epilogue (no separate add), every
    weight gradient on the side stream (reference: the torchvision blocks of ``imagenet.py:312``,
    backward ``:128``)."""

    @staticmethod
    def forward(ctx, x, block, ws):
        from .conv import deterministic
        fuse = not deterministic()
        pairs = block.convs_bns()
        h = x
        saved, saves = [x], []
        for conv, bn, _ in pairs[:-1]:
            a = _conv_bn_stats(h, conv, bn, fuse)
            h, sv = bn_train_f32(a, bn, ws, None, True)
            saved += [a, h]
            saves.append(sv)
        conv, bn, _ = pairs[-1]
        a = _conv_bn_stats(h, conv, bn, fuse)
        ds = block.downsample
        ad = svd = None
        idt = x
        if ds is not None:
            ad = _conv_bn_stats(x, ds[0], ds[1], fuse)
            idt, svd = bn_train_f32(ad, ds[1], ws, None, False)
        y, sv = bn_train_f32(a, bn, ws, idt, True)
        saves.append(sv)
        ctx.block, ctx.ws, ctx.n = block, ws, len(pairs)
        ctx.save_for_backward(*saved, a, ad, y, svd, *saves)
        return y

    @staticmethod
    def backward(ctx, g):
        from .conv import deterministic
        fuse = not deterministic()  # BN-backward reductions in the inner dgrads' epilogues
        t = ctx.saved_tensors
        n, block, ws = ctx.n, ctx.block, ctx.ws
        x = t[0]
        acts = [t[1 + 2 * i] for i in range(n - 1)]
        hs = [t[2 + 2 * i] for i in range(n - 1)]
        a_last, ad, y, svd = t[2 * n - 1], t[2 * n], t[2 * n + 1], t[2 * n + 2]
        saves = t[2 * n + 3:]
        pairs = block.convs_bns()
        ds = block.downsample
        g = g.contiguous()
        dA, dres = _bn_bwd(g, y, a_last, saves[-1], pairs[-1][1], ws, True)
        if ds is not None:
            dAd, _ = _bn_bwd(dres, None, ad, svd, ds[1], ws, False)
            dX = _dgrad(ds[0], dAd, x.shape)
            _wgrad_side(ds[0], dAd, x)
        else:
            dX = dres  # the identity branch's gradient; conv1's dgrad accumulates into it
        inputs = [x] + hs
        for i in range(n - 1, -1, -1):
            conv = pairs[i][0]
            if i > 0:
                bn_prev = pairs[i - 1][1]
                fused = False
                if fuse:
                    dH, fused = _dgrad(conv, dA, inputs[i].shape, bnb=(acts[i - 1], saves[i - 1], bn_prev))
                else:
                    dH = _dgrad(conv, dA, inputs[i].shape)
                _wgrad_side(conv, dA, inputs[i])
                if fused:  # dH is already masked; its reductions are in bn_prev's slab
                    dA = _bn_bwd_slab(dH, acts[i - 1], saves[i - 1], bn_prev, ws)
                else:
                    dA, _ = _bn_bwd(dH, hs[i - 1], acts[i - 1], saves[i - 1], bn_prev, ws, False)
            else:
                _dgrad(conv, dA, x.shape, out=dX, accumulate=True)
                _wgrad_side(conv, dA, x)
        return dX, None, None


# ------------------------------------------------------------------ pooling, loss, input
def maxpool_f32(x: torch.Tensor, k: int, s: int, p: int):
    N, H, W, Cc = x.shape
    OH, OW = conv_out_size(H, k, s, p), conv_out_size(W, k, s, p)
    y = torch.empty((N, OH, OW, Cc), device=x.device, dtype=torch.float32)
    idx = torch.empty((N, OH, OW, Cc), device=x.device, dtype=torch.uint8)
    _lib.check(_k().imk_maxpool_f32(x.data_ptr(), y.data_ptr(), idx.data_ptr(), N, H, W, Cc, OH, OW, k, s, p,
                                    _lib.stream_ptr()), "maxpool f32")
    return y, idx


class MaxPoolF32Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        y, idx = maxpool_f32(x, k, s, p)
        ctx.save_for_backward(idx)
        ctx.cfg = (tuple(x.shape), k, s, p)
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        (N, H, W, Cc), k, s, p = ctx.cfg
        OH, OW = idx.shape[1], idx.shape[2]
        dx = torch.empty((N, H, W, Cc), device=dy.device, dtype=torch.float32)
        _lib.check(_k().imk_maxpool_bwd_f32(dy.contiguous().data_ptr(), idx.data_ptr(), dx.data_ptr(), N, H, W, Cc,
                                            OH, OW, k, s, p, _lib.stream_ptr()), "maxpool bwd f32")
        return dx, None, None, None


def avgpool_f32(x: torch.Tensor) -> torch.Tensor:
    N, H, W, Cc = x.shape
    y = torch.empty((N, Cc), device=x.device, dtype=torch.float32)
    _lib.check(_k().imk_avgpool_f32(x.data_ptr(), y.data_ptr(), N, H * W, Cc, _lib.stream_ptr()), "avgpool f32")
    return y


class AvgPoolF32Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.shape = tuple(x.shape)
        return avgpool_f32(x)

    @staticmethod
    def backward(ctx, dy):
        N, H, W, Cc = ctx.shape
        dx = torch.empty(ctx.shape, device=dy.device, dtype=torch.float32)
        _lib.check(_k().imk_avgpool_bwd_f32(dy.contiguous().data_ptr(), dx.data_ptr(), N, H * W, Cc,
                                            _lib.stream_ptr()), "avgpool bwd f32")
        return dx


class XentF32Fn(torch.autograd.Function):
    """The fused softmax-xent (+ top-k counters) of ``ops.misc.XentFn`` with an fp32 logits gradient."""

    @staticmethod
    def forward(ctx, logits, labels, metrics, smoothing):
        from .misc import XentFn
        loss = XentFn.forward(ctx, logits, labels, metrics, smoothing)
        return loss

    @staticmethod
    def backward(ctx, gout):
        logits, labels, lse = ctx.saved_tensors
        B, NC = logits.shape
        dz = torch.empty((B, NC), device=logits.device, dtype=torch.float32)
        g = gout.to(torch.float32).contiguous()
        _lib.check(_k().imk_xent_bwd_f32(logits.data_ptr(), labels.data_ptr(), lse.data_ptr(), g.data_ptr(),
                                         dz.data_ptr(), B, NC, float(ctx.smoothing), _lib.stream_ptr()),
                   "xent bwd f32")
        return dz, None, None, None


def normalize_u8_f32(images: torch.Tensor, out_hw, cpad: int, mean: Sequence[float], std: Sequence[float],
                     crop: Optional[torch.Tensor] = None, flip: Optional[torch.Tensor] = None) -> torch.Tensor:
    """uint8 [B, Hs, Ws, 3] -> fp32 NHWC [B, H, W, cpad] (ToTensor + Normalize, imagenet.py:280-283)."""
    B, Hs, Ws, _ = images.shape
    H, W = out_hw
    out = torch.empty((B, H, W, cpad), device=images.device, dtype=torch.float32)
    m = (C.c_float * 3)(*mean)
    s = (C.c_float * 3)(*std)
    _lib.check(_k().imk_normalize_u8_f32(images.data_ptr(), out.data_ptr(), _lib.ptr(crop), _lib.ptr(flip), B, Hs,
                                         Ws, H, W, cpad, C.cast(m, C.c_void_p), C.cast(s, C.c_void_p),
                                         _lib.stream_ptr()), "normalize f32")
    return out
