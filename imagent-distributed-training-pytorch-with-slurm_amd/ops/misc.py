"""Pooling, loss + metrics, optimizer and input kernels (Python side)."""

from __future__ import annotations

import ctypes as C
from typing import Optional, Sequence

import torch

from . import _lib
from .conv import conv_out_size


# ----------------------------------------------------------------- pooling
class MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        N, H, W, Cc = x.shape
        OH, OW = conv_out_size(H, k, s, p), conv_out_size(W, k, s, p)
        y = torch.empty((N, OH, OW, Cc), device=x.device, dtype=x.dtype)
        idx = torch.empty((N, OH, OW, Cc), device=x.device, dtype=torch.uint8)
        _lib.check(_lib.kernels().imk_maxpool_fwd(x.data_ptr(), y.data_ptr(), idx.data_ptr(), N, H, W,
                                                  Cc, OH, OW, k, s, p, _lib.stream_ptr()), "maxpool")
        ctx.save_for_backward(idx)
        ctx.geom = (N, H, W, Cc, OH, OW, k, s, p)
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        N, H, W, Cc, OH, OW, k, s, p = ctx.geom
        dx = torch.empty((N, H, W, Cc), device=dy.device, dtype=torch.bfloat16)
        _lib.check(_lib.kernels().imk_maxpool_bwd(dy.contiguous().data_ptr(), idx.data_ptr(),
                                                  dx.data_ptr(), N, H, W, Cc, OH, OW, k, s, p,
                                                  _lib.stream_ptr()), "maxpool bwd")
        return dx, None, None, None


class BNReluPoolFn(torch.autograd.Function):
    """y = maxpool(relu(bn(x))) for the stem, fused both ways: the forward pools
    bf16(relu(bn(x))) straight from the BN input (``imk_maxpool_fwd_bn``: the
    BN output is never written), the backward stores the ReLU-masked BN
    upstream gradient and reduces the BN-backward sums in the same pass
    (``imk_maxpool_bwd_bnr``), then one BN apply pass -- instead of BN forward
    + pool forward and pool backward + BN reduce + BN apply.
    Reference ops: torchvision resnet ``bn1 -> relu -> maxpool``
    (/root/reference/imagenet.py:312)."""

    @staticmethod
    def forward(ctx, x, bn, k, s, p):
        from .bn import stats_finalize
        N, H, W, Cc = x.shape
        OH, OW = conv_out_size(H, k, s, p), conv_out_size(W, k, s, p)
        y = torch.empty((N, OH, OW, Cc), device=x.device, dtype=x.dtype)
        idx = torch.empty((N, OH, OW, Cc), device=x.device, dtype=torch.uint8)
        w = bn.work
        stats_finalize(w, N * H * W)  # conv-epilogue slab -> (mean, var) (also read by the running-stat update)
        _lib.check(_lib.kernels().imk_maxpool_fwd_bn(
            x.data_ptr(), w.stats.data_ptr(), bn.weight.data_ptr(), bn.bias.data_ptr(), w.save.data_ptr(),
            y.data_ptr(), idx.data_ptr(), None, N, H, W, Cc, OH, OW, k, s, p, bn.eps, _lib.stream_ptr()),
            "bn + maxpool")
        ctx.save_for_backward(x, idx)
        ctx.bn = bn
        ctx.geom = (N, H, W, Cc, OH, OW, k, s, p)
        return y

    @staticmethod
    def backward(ctx, dy):
        from .bn import bn_apply_backward
        x, idx = ctx.saved_tensors
        bn = ctx.bn
        N, H, W, Cc, OH, OW, k, s, p = ctx.geom
        g = torch.empty((N, H, W, Cc), device=dy.device, dtype=torch.bfloat16)
        w = bn.work
        _lib.check(_lib.kernels().imk_maxpool_bwd_bnr(
            dy.contiguous().data_ptr(), idx.data_ptr(), g.data_ptr(), x.data_ptr(), None, w.save.data_ptr(),
            bn.weight.data_ptr(), bn.bias.data_ptr(), w.scratch.data_ptr(), N, H, W, Cc, OH, OW, k, s, p,
            _lib.stream_ptr()), "maxpool bwd + bn reduce")
        dx, _ = bn_apply_backward(g, x, None, bn, None, 0)
        from . import streams
        streams.flush_deferred()  # layer1's conv1 weight gradient, after this BN pass
        return dx, None, None, None, None


class StemFn(torch.autograd.Function):
    """The 224-px stem -- conv1 (7x7 / 2) -> bn1 -> ReLU -> maxpool -- as ONE autograd node, so that the stem BN's
    backward apply pass never runs: the pool backward stores the ReLU-masked gradient g and reduces the BN sums
    (as BNReluPoolFn), ``imk_bn_bwd_coef`` turns them into dx = A g + B x + c (and dgamma / dbeta), and the stem's
    band weight gradient applies that on its operand staging (``ops.conv.stem_wgrad_bnx``) -- the stem conv's
    input (the image) needs no gradient, so dx is never materialised (one read of g and x and one write of dx
    less: 3 x 3.3 GB at 2048 img/GPU). Reference ops: torchvision resnet ``conv1 -> bn1 -> relu -> maxpool``
    (/root/reference/imagenet.py:312, backward :128)."""

    @staticmethod
    def forward(ctx, img, weight, conv, bn, k, s, p):
        from .bn import stats_finalize
        from .conv import igemm_fwd
        x = igemm_fwd(img, conv.w_bf16, conv.stride, conv.padding, conv.kh, conv.kw, stats=bn.work, stem=True)
        N, H, W, Cc = x.shape
        OH, OW = conv_out_size(H, k, s, p), conv_out_size(W, k, s, p)
        y = torch.empty((N, OH, OW, Cc), device=x.device, dtype=x.dtype)
        idx = torch.empty((N, OH, OW, Cc), device=x.device, dtype=torch.uint8)
        # the BN input at each window's argmax: the pool backward's ReLU mask and BN sums come from it
        # instead of a read of x (4x its bytes): pool backward 2,034 -> 1,772 us, pool forward 1,052 -> 1,167 us
        # at 2048 img; in-step 17,130 / 17,181 vs 17,091 / 17,169 img/s (same box)
        xsel = torch.empty_like(y)
        w = bn.work
        stats_finalize(w, N * H * W)
        _lib.check(_lib.kernels().imk_maxpool_fwd_bn(
            x.data_ptr(), w.stats.data_ptr(), bn.weight.data_ptr(), bn.bias.data_ptr(), w.save.data_ptr(),
            y.data_ptr(), idx.data_ptr(), xsel.data_ptr(), N, H, W, Cc, OH, OW, k, s, p, bn.eps,
            _lib.stream_ptr()), "bn + maxpool")
        ctx.save_for_backward(img, x, idx, xsel)
        ctx.mods = (conv, bn)
        ctx.geom = (N, H, W, Cc, OH, OW, k, s, p)
        return y

    @staticmethod
    def backward(ctx, dy):
        from . import streams
        from .conv import stem_wgrad_bnx
        from .grad_sink import notify_ready
        img, x, idx, xsel = ctx.saved_tensors
        conv, bn = ctx.mods
        N, H, W, Cc, OH, OW, k, s, p = ctx.geom
        g = torch.empty((N, H, W, Cc), device=dy.device, dtype=torch.bfloat16)
        w = bn.work
        kern = _lib.kernels()
        _lib.check(kern.imk_maxpool_bwd_bnr(
            dy.contiguous().data_ptr(), idx.data_ptr(), g.data_ptr(), x.data_ptr(), xsel.data_ptr(), w.save.data_ptr(),
            bn.weight.data_ptr(), bn.bias.data_ptr(), w.scratch.data_ptr(), N, H, W, Cc, OH, OW, k, s, p,
            _lib.stream_ptr()), "maxpool bwd + bn reduce")
        coef = torch.empty((3, Cc), device=dy.device, dtype=torch.float32)
        _lib.check(kern.imk_bn_bwd_coef(w.scratch.data_ptr(), w.save.data_ptr(), bn.weight.data_ptr(),
                                        bn.weight.grad.data_ptr(), bn.bias.grad.data_ptr(), coef.data_ptr(),
                                        N * H * W, Cc, _lib.stream_ptr()), "stem bn bwd coef")
        notify_ready(bn.weight)
        notify_ready(bn.bias)
        streams.flush_deferred()  # layer1's conv1 weight gradient (queued behind this BN's backward)
        side = streams.side_stream(dy.device)
        if side is not None:
            streams.wait(side, torch.cuda.current_stream(dy.device))
        with torch.cuda.stream(side) if side is not None else _NullCtx():
            gp = conv.grad_pad
            ok = stem_wgrad_bnx(g, img, gp, x, coef, conv.stride, conv.padding, conv.kh, conv.kw)
            assert ok, "StemFn needs the band stem's shape (models.native checks it)"
            gw = conv.weight.grad
            _lib.check(kern.imk_stem_grad_fold(gp.data_ptr(), gw.data_ptr(), gp.shape[0], conv.in_channels,
                                               conv.kh, conv.kw, _lib.stream_ptr()), "stem grad fold")
            notify_ready(conv.weight)
        if side is not None:
            streams.protect(g, img, x, coef)
            streams.ensure_join_after_backward()
        return None, None, None, None, None, None, None


class _NullCtx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def stem_fused_ok(img: torch.Tensor, conv) -> bool:
    """Does StemFn cover this stem (the band kernels' shape: 224-px 4-channel input, 7x7 / 2 / 3, 64 channels)?"""
    return (img.dim() == 4 and img.shape[1] == 224 and img.shape[2] == 224 and img.shape[3] == 4 and
            conv.kh == 7 and conv.kw == 7 and conv.stride == 2 and conv.padding == 3 and conv.out_channels == 64 and
            getattr(conv, "grad_pad", None) is not None)


def maxpool_eval(x, k, s, p):
    N, H, W, Cc = x.shape
    OH, OW = conv_out_size(H, k, s, p), conv_out_size(W, k, s, p)
    y = torch.empty((N, OH, OW, Cc), device=x.device, dtype=x.dtype)
    _lib.check(_lib.kernels().imk_maxpool_fwd(x.data_ptr(), y.data_ptr(), None, N, H, W, Cc, OH, OW,
                                              k, s, p, _lib.stream_ptr()), "maxpool")
    return y


class AvgPoolFn(torch.autograd.Function):
    """Global average pool NHWC [N,H,W,C] -> [N,C] (AdaptiveAvgPool2d((1,1)) + flatten)."""

    @staticmethod
    def forward(ctx, x):
        N, H, W, Cc = x.shape
        y = torch.empty((N, Cc), device=x.device, dtype=x.dtype)
        _lib.check(_lib.kernels().imk_avgpool_fwd(x.data_ptr(), y.data_ptr(), N, H * W, Cc,
                                                  _lib.stream_ptr()), "avgpool")
        ctx.shape = (N, H, W, Cc)
        return y

    @staticmethod
    def backward(ctx, dy):
        N, H, W, Cc = ctx.shape
        dx = torch.empty((N, H, W, Cc), device=dy.device, dtype=torch.bfloat16)
        _lib.check(_lib.kernels().imk_avgpool_bwd(dy.to(torch.bfloat16).contiguous().data_ptr(),
                                                  dx.data_ptr(), N, H * W, Cc, _lib.stream_ptr()),
                   "avgpool bwd")
        return dx


# ------------------------------------------------------------ loss+metrics
class XentFn(torch.autograd.Function):
    """Mean softmax cross-entropy (nn.CrossEntropyLoss, imagenet.py:323) with
    fused top-1/top-5 counting into a device metrics vector
    ``[loss_sum, top1_hits, top5_hits, rows]`` - no host sync per step."""

    @staticmethod
    def forward(ctx, logits, labels, metrics, smoothing):
        logits = logits.contiguous()
        B, NC = logits.shape
        lse = torch.empty(B, device=logits.device, dtype=torch.float32)
        loss = torch.empty((), device=logits.device, dtype=torch.float32)  # cleared by imk_xent_fwd
        _lib.check(_lib.kernels().imk_xent_fwd(logits.data_ptr(), labels.data_ptr(), lse.data_ptr(),
                                               loss.data_ptr(), _lib.ptr(metrics), B, NC,
                                               float(smoothing), _lib.stream_ptr()), "xent")
        ctx.save_for_backward(logits, labels, lse)
        ctx.smoothing = smoothing
        return loss

    @staticmethod
    def backward(ctx, gout):
        logits, labels, lse = ctx.saved_tensors
        B, NC = logits.shape
        g = gout.to(torch.float32).contiguous()
        # the logits' own dtype (fp32): autograd would otherwise cast a bf16 gradient back with an ATen copy; the
        # linear layer's backward rounds it to bf16 with its own kernel
        dz = torch.empty((B, NC), device=logits.device, dtype=logits.dtype)
        fn = _lib.kernels().imk_xent_bwd_f32 if logits.dtype == torch.float32 else _lib.kernels().imk_xent_bwd
        _lib.check(fn(logits.data_ptr(), labels.data_ptr(), lse.data_ptr(), g.data_ptr(), dz.data_ptr(), B, NC,
                      float(ctx.smoothing), _lib.stream_ptr()), "xent bwd")
        return dz, None, None, None


# -------------------------------------------------------------------- SGD
def sgd_flat(p: torch.Tensor, g: torch.Tensor, buf: Optional[torch.Tensor],
             shadow: Optional[torch.Tensor], lr: float, momentum: float, dampening: float,
             weight_decay: float, nesterov: bool, first: bool, grad_scale: float = 1.0) -> None:
    _lib.check(_lib.kernels().imk_sgd(p.data_ptr(), g.data_ptr(), _lib.ptr(buf), _lib.ptr(shadow),
                                      p.numel(), lr, momentum, dampening, weight_decay,
                                      1 if nesterov else 0, 1 if first else 0, grad_scale,
                                      _lib.stream_ptr()), "sgd")


def cast_bf16(src: torch.Tensor, dst: torch.Tensor) -> None:
    _lib.check(_lib.kernels().imk_cast_bf16(src.data_ptr(), dst.data_ptr(), src.numel(),
                                            _lib.stream_ptr()), "cast")


def uncast_bf16(src: torch.Tensor, dst: torch.Tensor) -> None:
    """bf16 ``src`` -> fp32 ``dst`` (same numel) on the current stream."""
    _lib.check(_lib.kernels().imk_uncast_bf16(src.data_ptr(), dst.data_ptr(), src.numel(),
                                              _lib.stream_ptr()), "uncast")


class TransposePlan:
    """Batched ``[Co][T][Ci] -> [Ci][T][Co]`` re-layout of every conv's bf16
    weight shadow into its dgrad shadow: one launch per optimizer step."""

    def __init__(self, items: Sequence[tuple], device):
        descs = (_lib.TDesc * max(1, len(items)))()
        tile = 0
        for i, (src, dst, Co, T, Ci) in enumerate(items):
            descs[i].src, descs[i].dst = src.data_ptr(), dst.data_ptr()
            descs[i].Co, descs[i].T, descs[i].Ci, descs[i].tile0 = Co, T, Ci, tile
            tile += ((Co + 31) // 32) * ((Ci + 31) // 32) * T
        raw = bytes(memoryview(descs))[: C.sizeof(_lib.TDesc) * len(items)]
        self.n = len(items)
        self.tiles = tile
        self.desc = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(device) if items else None

    def run(self) -> None:
        if self.n:
            _lib.check(_lib.kernels().imk_transpose_batched(self.desc.data_ptr(), self.n, self.tiles,
                                                            _lib.stream_ptr()), "transpose")


# -------------------------------------------------------------- normalize
def resize_normalize_u8(images: torch.Tensor, out_hw, cpad: int, mean: Sequence[float], std: Sequence[float],
                        flip: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """uint8 [B, Hs, Ws, 3] -> bf16 NHWC [B, H, W, cpad]: bilinear resample to (H, W) (half-pixel centres,
    ``F.interpolate(mode='bilinear', align_corners=False)``) fused with (x/255 - mean)/std -- the records stored
    smaller than the model input (``--record-resize``), resized on the GPU instead of on the host
    (imagenet.py:281's Resize, moved after the gather)."""
    B, Hs, Ws, _ = images.shape
    H, W = out_hw
    if out is None:
        out = torch.empty((B, H, W, cpad), device=images.device, dtype=torch.bfloat16)
    m = (C.c_float * 3)(*mean)
    s = (C.c_float * 3)(*std)
    _lib.check(_lib.kernels().imk_resize_normalize_u8(images.data_ptr(), out.data_ptr(), _lib.ptr(flip), B, Hs, Ws,
                                                      H, W, cpad, C.cast(m, C.c_void_p), C.cast(s, C.c_void_p),
                                                      _lib.stream_ptr()), "resize + normalize")
    return out


def normalize_u8(images: torch.Tensor, out_hw, cpad: int, mean: Sequence[float], std: Sequence[float],
                 crop: Optional[torch.Tensor] = None, flip: Optional[torch.Tensor] = None,
                 out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """uint8 [B, Hs, Ws, 3] -> bf16 NHWC [B, H, W, cpad]: (x/255 - mean)/std
    (ToTensor + Normalize of imagenet.py:280-283, on the GPU)."""
    B, Hs, Ws, _ = images.shape
    H, W = out_hw
    if out is None:
        out = torch.empty((B, H, W, cpad), device=images.device, dtype=torch.bfloat16)
    m = (C.c_float * 3)(*mean)
    s = (C.c_float * 3)(*std)
    _lib.check(_lib.kernels().imk_normalize_u8(images.data_ptr(), out.data_ptr(), _lib.ptr(crop),
                                               _lib.ptr(flip), B, Hs, Ws, H, W, cpad,
                                               C.cast(m, C.c_void_p), C.cast(s, C.c_void_p),
                                               _lib.stream_ptr()), "normalize")
    return out
