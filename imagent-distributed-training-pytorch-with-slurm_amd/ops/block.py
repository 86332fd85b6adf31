"""One autograd node per residual block with a hand-scheduled backward.

torchvision's BasicBlock / Bottleneck (reference model, ``imagenet.py:312``)
become a single :class:`BlockFn` on the HIP path. Forward runs the block's
kernels back to back (conv with BN statistics in its epilogue -> fused
BN+ReLU, ..., last conv -> fused BN + shortcut (+ downsample BN) + ReLU).
The backward is explicit instead of autograd-derived, which lets it

* fuse the residual fan-in: the shortcut gradient (masked upstream gradient
  or the downsample conv's dgrad) is written first and the block's first conv
  ACCUMULATES its dgrad into it in the GEMM epilogue (no separate add kernel,
  no extra read/write of a full activation);
* release each parameter's gradient to the bucketed reducer the moment its
  kernel has been queued (bn3 -> conv3 -> bn2 -> conv2 -> bn1 -> ds -> conv1);
* skip the ReLU-output read in BN backward (mask recomputed from x);
* fold each BatchNorm-backward reduction into the dgrad that produces the
  BN's upstream gradient (``BNBwdFuse``, conv epilogue IG_BNBWD): the dgrad
  stores the ReLU-masked gradient and adds sum(g), sum(g*xhat) to the BN's
  slab, so BN backward is a single apply pass. Inside a block this covers
  bn1..bnK-1; the block's LAST BN is finished by the NEXT block's first-conv
  dgrad (the last writer of this block's output gradient, `_prev_block`
  link), which marks it `_bnb_done`.

It also removes ~6 autograd nodes and their Python dispatch per block.
"""

from __future__ import annotations

import os

import torch

from . import _lib, streams
from . import conv as _conv
from .bn import bn_act_backward, bn_act_forward, bn_apply_backward, bn_scale_shift
from .bn_gram import GramBN, gram_T, gram_coef, gram_dgrad, gram_fwd_stats, gram_wgrad
from .conv import BNBwdFuse, conv_wgrad, igemm_dgrad, igemm_fwd


# Each weight gradient is issued after the BN-backward pass that follows its dgrad, so the side stream's wgrad
# overlaps the next (compute-bound) dgrad rather than the memory-bound BN pass (the two passes sharing HBM slowed
# the BN pass from 13 to 23 ms/step): measured +1.1 % img/s at R50 / 1024 (12,131 vs 12,001). The downsample
# conv's forward runs on the side stream beside the main chain's BN passes, and a stride-2 1x1 downsample dgrad
# writes only the pixels it reaches (no memset; conv1's accumulating dgrad knows the rest are zero).
# IMAGENT_BN_XFUSE (default 1; 0 = A/B off): a BatchNorm + ReLU inside a block whose consumer conv can
# take it on its operand path is not a pass of its own: its statistics are finalized into a per-channel
# scale / shift and the consumer applies them (+ ReLU) on its operand load -- the streaming 1x1 conv
# (a bottleneck's conv3 with K = 64 / 128) or the halo-tiled 64 -> 64 3x3 conv (the stage-1 conv2 of
# ResNet-50 at 56x56, of ResNet-18/34 at 56x56 / 112x112) -- and its weight gradient on the operand
# staging (ops/conv.py xbn); the BN output is never written or read. Measured at R50 / 1024 with the
# 1x1 consumers: +0.43 % img/s (12,499 / 12,497 vs 12,446 / 12,440, same box)
# (IMAGENT_BN_XFUSE=all: also the halo 3x3 consumers -- numerics-tested, measured -0.3 % at R50 / 1024 and
# R18 448^2: the patch staging's extra VALU costs more than the skipped pass saves; opt-in)
_XFUSE = os.environ.get("IMAGENT_BN_XFUSE", "1") != "0"
_XFUSE_3X3 = os.environ.get("IMAGENT_BN_XFUSE", "1") == "all"
# IMAGENT_BN_GRAM (default 1; 0 = A/B off): a bottleneck's last BatchNorm backward without its apply pass
# (ops/bn_gram.py): conv3's dgrad runs over [g | h2] with folded weights, its wgrad from g^T h2 and the
# Gram matrix of h2. conv3's input h2 is then kept (no operand-path BN fusion for that conv).
_GRAM = os.environ.get("IMAGENT_BN_GRAM", "1") != "0"
# with it, the next block's conv1 dgrad does not read x3 for bn3's sum(g xhat): x3 = h2 W3^T, so that sum is
# rowsum(W3 * g^T h2) -- the weight gradient's GEMM (IMAGENT_BN_GRAM=slab: from the epilogue's x3 read, A/B)
_GRAM_NOX = os.environ.get("IMAGENT_BN_GRAM", "1") != "slab"
# ... for blocks with at least this many output pixels (N x OH x OW): the form saves ~32 M p bytes of BatchNorm
# traffic per block but costs two p x p x M GEMM extensions and ~8 small launches, so below ~10^5 pixels it
# loses (same-box A/B: ResNet-152 at 256 img/GPU 4,699 img/s with every block in the Gram form vs 5,080 without,
# at 1024 img/GPU 6,279 vs 6,019; ResNet-50 at 256 11,636 vs 12,097)
_GRAM_MIN_ROWS = int(os.environ.get("IMAGENT_GRAM_MIN_ROWS", "100000"))
# the downsample conv's forward on the main stream (default) or, IMAGENT_DS_SIDE=1, on the side stream beside the
# main chain's BN passes (rounds 2-5): at 4096 img the side placement lost in 5 of 5 alternating pairs, +0.1-1.0 %
# for the main stream (scripts/runs/ds_ab.sh, ds_ab2.sh; profiles/ab/ds_side_r6.txt) -- the side stream's
# concurrent work slows the memory-bound main-chain kernels more than the overlap gains (profiles/
# instep_contention_r6.md); neutral at 256 img
_DS_SIDE = os.environ.get("IMAGENT_DS_SIDE", "0") == "1"
# ... and bottleneck widths p <= 256: the extension grows as p^2 M against ~32 M p bytes saved, and at p = 512
# (ResNet-50's layer 4) it loses at the same per-block work where p = 256 wins (same-box A/B at 2048 img/GPU, where
# layer 4 passes the row bound: 16,620 / 16,610 img/s without its Gram form vs 16,543 / 16,529 with it; layer 3 at
# 1024 img, the same M p, is a round-4 win)
_GRAM_MAX_P = 256
# ... and in identity blocks bn3's FORWARD too: its batch statistics come from h2 (mean = W3 colsum(h2) / M,
# E[x3^2] = rowsum(W3 G * W3) / M with the Gram matrix G the weight gradient needs anyway), so conv3's epilogue
# applies bn3 + shortcut + ReLU and writes the block output and its mask bits: x3 is never written or read
# (IMAGENT_BN_GRAM_FWD=0: off, A/B)
_GRAM_FWD = os.environ.get("IMAGENT_BN_GRAM_FWD", "1") != "0"


def _gram_ok(block, q, x) -> bool:
    """Does this block's backward take bn3 through the Gram form (forward keeps h2)?"""
    pairs = block.convs_bns()
    if not (_GRAM and x.is_cuda and len(pairs) == 3):  # (with fp8: conv3's dgrad stays bf16 in this form)
        return False
    if _conv.deterministic():  # split-K atomics accumulate G / T: never on the bit-identical statistics path
        return False
    if not getattr(block, "_fuse_bnb", False):  # the next block's dgrad must reduce bn3 (premasked backward)
        return False
    c3 = pairs[-1][0]
    s = pairs[1][0].stride  # the bottleneck's stride sits in conv2
    rows = x.shape[0] * (x.shape[1] // s) * (x.shape[2] // s)
    return (c3.kh == 1 and c3.kw == 1 and c3.stride == 1 and c3.padding == 0 and c3.in_channels % 64 == 0
            and c3.out_channels % 64 == 0 and rows >= _GRAM_MIN_ROWS
            and (c3.in_channels <= _GRAM_MAX_P or _GRAM_MIN_ROWS == 0))


def _xfuse_ok(conv, a, q) -> bool:
    """Can ``conv`` (the consumer of BN(a) + ReLU) apply that BN on its operand path?"""
    if not (_XFUSE and (q is None or not fp8_fwd_ok(conv)) and a.is_cuda) or _conv._NOSTREAM:
        return False
    if conv.kh == 1 and conv.kw == 1:
        return (conv.stride == 1 and conv.padding == 0 and conv.in_channels in (64, 128)
                and conv.out_channels % 128 == 0)
    H, W = a.shape[1], a.shape[2]
    # the halo kernel's launch conditions (conv_halo.hip, conv_halo()): W 56 with H % 4 == 0, or W 112 with
    # H % 2 == 0
    return (_XFUSE_3X3 and conv.kh == 3 and conv.kw == 3 and conv.stride == 1 and conv.padding == 1
            and conv.in_channels == 64 and conv.out_channels == 64
            and ((W == 56 and H % 4 == 0) or (W == 112 and H % 2 == 0)))


def _fwd(conv, h, bn):
    return igemm_fwd(h, conv.w_bf16, conv.stride, conv.padding, conv.kh, conv.kw,
                     stats=bn.work, stem=getattr(conv, "stem", False))


# --dtype fp8 runs a conv on the 1-byte v3 loop only where that measured faster than the bf16 kernels
# (per-shape table: profiles/r50_b1024_fp8_v3_kernel_stats.md); everywhere else, and for everything the bf16
# path fuses (operand-path BN, the Gram-form bn3 backward), the step stays bf16 and no fp8 copy is written.
def fp8_fwd_ok(conv) -> bool:
    """Forward on fp8: 3x3 with >= 128 input channels, 1x1 with >= 512, or 256 into <= 128 channels (the
    1x1 convs with K <= 256 into wide outputs are HBM streams the bf16 streaming kernel runs faster)."""
    ci, co = conv.in_channels, conv.out_channels
    if conv.kh > 1:
        return ci >= 128
    return ci >= 512 or (ci == 256 and co <= 128)


def fp8_dgrad_ok(conv) -> bool:
    """dgrad on fp8 (it gathers over the gradient's out_channels): 3x3 with >= 128, 1x1 with >= 512, or 256
    into <= 128 input channels (256 into wider: the bf16 streaming BN-backward dgrad wins)."""
    ci, co = conv.in_channels, conv.out_channels
    if conv.kh > 1:
        return co >= 128
    return co >= 512 or (co == 256 and ci <= 128)


def _fwd8(conv, h, h8, bn):
    """fp8 forward (``Fp8State``) when the input has an e4m3 copy and the shape is one fp8 wins, else bf16."""
    if h8 is None or conv.in_channels % 16 or not fp8_fwd_ok(conv):
        return _fwd(conv, h, bn)
    return igemm_fwd(h8[0], conv.w8, conv.stride, conv.padding, conv.kh, conv.kw, stats=bn.work,
                     fp8=(h8[1], conv.w8_exp))


def _use8(q, g8):
    """The e5m2 copy a BN-backward pass wrote, once gradient scales exist."""
    return (g8[0], g8[1]) if (g8 is not None and q.grad_ready) else None


def _dg8(d8, conv):
    """fp8 dgrad operands (e5m2 gradient, e4m3 transposed weights) or None (bf16)."""
    if d8 is None or getattr(conv, "wt8", None) is None or conv.out_channels % 16 or not fp8_dgrad_ok(conv):
        return None
    return (d8[0], d8[1], conv.wt8, conv.w8_exp)


def _gws(block, i):
    """Entry i (0 T, 1 G, 2 colsum, 3 Q, 4 P) of the block's zeroed Gram workspace, or None (allocated on demand)."""
    w = getattr(block, "_gram_ws", None)
    return w[i] if w is not None else None


def _wgrad(conv, dA, h):
    """``h`` is the conv's input, or (BN input, scale / shift) when the BN + ReLU before it is
    applied on the operand path (``IMAGENT_BN_XFUSE``)."""
    if isinstance(h, tuple):
        conv_wgrad(conv, dA, h[0], xbn=h[1])
    else:
        conv_wgrad(conv, dA, h)


class BlockFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, block):
        pairs = block.convs_bns()
        q = getattr(block, "_q8", None)  # Fp8State or None
        if q is not None and not q.active:
            q = None  # not inside a forward_hip training pass
        x8 = q.lookup(x) if q is not None else None
        saved = [x]
        h, h8 = x, x8
        ds = block.downsample
        # the downsample conv depends only on x: with IMAGENT_DS_SIDE=1 it runs on the (idle in forward) side stream
        # beside the main chain's memory-bound BN passes (off by default, see _DS_SIDE)
        side = streams.side_stream(x.device) if (ds is not None and x.is_cuda and _DS_SIDE) else None
        ad = None
        if side is not None:
            streams.wait(side, torch.cuda.current_stream())
            with torch.cuda.stream(side):
                ad = _fwd8(ds[0], x, x8, ds[1])
        xbn = [None] * len(pairs)  # xbn[i]: conv i applies the preceding BN + ReLU on its operand load
        gram = _gram_ok(block, q, x)  # bn3 backward in the Gram form: conv3's input must exist
        ss = None
        h2sum = None  # Gram form: colsum(h2), accumulated by the BN pass that writes h2
        for i, (conv, bn, _) in enumerate(pairs[:-1]):
            a = _fwd8(conv, h, h8, bn) if ss is None else \
                igemm_fwd(h, conv.w_bf16, conv.stride, conv.padding, conv.kh, conv.kw, stats=bn.work, xbn=ss)
            ss = None
            if not (gram and i + 1 == len(pairs) - 1) and _xfuse_ok(pairs[i + 1][0], a, q):
                ss = xbn[i + 1] = bn_scale_shift(a, bn)
                h, h8 = a, None
                saved += [a, None]
                continue
            q8 = q.out_for(a, q.slot[id(bn)]) if (q is not None and fp8_fwd_ok(pairs[i + 1][0])) else None
            if gram and i + 1 == len(pairs) - 1:
                gws = getattr(block, "_gram_ws", None)  # zeroed per step with the BN slabs (models/native.py)
                h2sum = gws[2] if gws is not None else torch.zeros(a.shape[-1], device=a.device,
                                                                    dtype=torch.float32)
            h = bn_act_forward(a, None, bn, None, 0, True, q8=q8, colsum=h2sum)
            h8 = (q8[0], q8[1]) if q8 is not None else None
            saved += [a, h]
        conv, bn, _ = pairs[-1]
        fuse_next = getattr(block, "_fuse_bnb", False)
        # the block output's e4m3 copy only when the next block's conv1 or downsample conv reads fp8
        need8 = q is not None and getattr(block, "_q8_out", True)
        gws = getattr(block, "_gram_ws", None)
        # bn3 + shortcut + ReLU in conv3's epilogue (x3 never materialised): a Gram-form block whose output mask
        # the next block's x-free dgrad epilogue reads, conv3 on the streaming kernel. A downsample block's
        # shortcut BN enters as a per-channel scale on the residual (its shift folded into bn3's)
        # (the fused-output epilogue exists only on the streaming kernel: not with IMAGENT_CONV_STREAM=0)
        fused3 = (gram and _GRAM_FWD and _GRAM_NOX and fuse_next and not _conv._NOSTREAM
                  and getattr(block, "_has_next", False) and gws is not None and h2sum is not None
                  and conv.in_channels in (64, 128, 256) and (ds is not None or x.shape[-1] == conv.out_channels))
        gram_P = None
        if fused3:
            res, rsc, ssd = x, None, None
            if ds is not None:
                if side is not None:
                    cur = torch.cuda.current_stream()
                    streams.wait(cur, side)
                    ad.record_stream(cur)
                else:
                    ad = _fwd8(ds[0], x, x8, ds[1])
                ssd = bn_scale_shift(ad, ds[1])
                res, rsc = ad, ssd[0]
            aff, gram_P = gram_fwd_stats(bn, conv, h, h2sum, gws[1], add_shift=ssd[1] if ssd is not None else None,
                                         P=gws[4])
            out = torch.empty(res.shape, device=res.device, dtype=res.dtype)
            # the ReLU mask of the block output as bits, for the next block's conv1 dgrad epilogue; the output's
            # e4m3 copy from the same epilogue when an fp8 conv reads it
            ym = torch.empty(out.numel() // 8, device=out.device, dtype=torch.uint8)
            q8 = q.out_for(out, q.slot[id(bn)]) if need8 else None
            igemm_fwd(h, conv.w_bf16, 1, 0, 1, 1, out=out, affine=aff, relu=True, res=res, maskout=ym, res_scale=rsc,
                      q8out=q8)
            a = None
        elif ss is not None:
            a = igemm_fwd(h, conv.w_bf16, conv.stride, conv.padding, conv.kh, conv.kw, stats=bn.work, xbn=ss)
        else:
            a = _fwd8(conv, h, h8, bn)
        if not fused3:
            q8 = q.out_for(a, q.slot[id(bn)]) if need8 else None
            # the ReLU mask of the block output as bits, for the next block's conv1 dgrad epilogue (1/16
            # of the bytes of re-reading the output there)
            ym = torch.empty(a.numel() // 8, device=a.device, dtype=torch.uint8) if fuse_next else None
        if fused3:
            pass
        elif ds is not None:
            if side is not None:
                cur = torch.cuda.current_stream()
                streams.wait(cur, side)
                ad.record_stream(cur)  # allocated on the side stream, read / freed in main order
            else:
                ad = _fwd8(ds[0], x, x8, ds[1])
            out = bn_act_forward(a, ad, bn, ds[1], 2, True, q8=q8, ym=ym)
        else:
            ad = None
            out = bn_act_forward(a, x, bn, None, 1, True, q8=q8, ym=ym)
        if q is not None:
            q.register(out, q8)
        saved += [a, ad, out]
        # rows seen by each BN (module order: bn1..bnK, downsample.1) for the running-stat update
        rows = [t.numel() // t.shape[-1] for t in saved[1:-3:2]] + [out.numel() // out.shape[-1]]
        if ad is not None:
            rows.append(ad.numel() // ad.shape[-1])
        block._bn_rows = rows
        # what the next block's backward needs to finish this block's last BN
        block._last_bn = (a, ad, ym) if fuse_next else None
        block._bnb_done = False
        ctx.block = block
        ctx.xbn = xbn
        ctx.gram = gram
        ctx.h2sum = h2sum
        ctx.gram_P = gram_P  # W3 G from the fused forward (G in the block's workspace): not recomputed
        block._gram = gram  # the next block's conv1 dgrad may then skip reading x3 (BNBwdFuse without x)
        block._bnb_nox = False
        ctx.save_for_backward(*saved)
        return out

    @staticmethod
    def backward(ctx, dout):
        block = ctx.block
        pairs = block.convs_bns()
        q = getattr(block, "_q8", None)  # Fp8State: e5m2 BN-backward outputs feed fp8 dgrads
        if q is not None and not q.backward:
            q = None
        t = ctx.saved_tensors
        x = t[0]
        n = len(pairs)
        # t = [x, a0, r0, a1, r1, ..., a_last, ad, out]; conv i's input is x (i=0) or r_{i-1}
        acts = [t[1 + 2 * i] for i in range(n - 1)]
        outs = [t[2 + 2 * i] for i in range(n - 1)]
        a_last, ad, out = t[-3], t[-2], t[-1]
        inputs = [x] + outs
        dout = dout.contiguous()
        H, W = x.shape[1], x.shape[2]
        conv_l, bn_l, _ = pairs[-1]
        ds = block.downsample
        fuse = getattr(block, "_fuse_bnb", False)
        premasked = getattr(block, "_bnb_done", False)
        dA8 = None
        sparse = False
        if ds is not None:
            if premasked and ctx.gram and fuse:
                # bn3 in the Gram form (as for identity blocks below); the downsample BN alone gets an apply pass:
                # its reductions (sum g, sum g xhat_d) sit in bn3's slab rows 1, 2 (read there, sgx_row=2)
                T = gram_T(dout, outs[-1], out=_gws(block, 0)) if getattr(block, "_bnb_nox", False) else None
                dA = gram_coef(bn_l, dout, T=T, w3=conv_l.w_bf16 if T is not None else None, hs=ctx.h2sum)
                dAd, _ = bn_apply_backward(dout, ad, None, ds[1], None, 1, slab_of=bn_l, sgx_row=2)
                dAd8 = None
            elif premasked:  # dout already masked + reduced by the next block's conv1 dgrad
                g8a = q.grad_out(a_last, bn_l) if (q is not None and fp8_dgrad_ok(conv_l)) else None
                g8b = q.grad_out(ad, ds[1]) if (q is not None and fp8_dgrad_ok(ds[0])) else None
                dA, dAd = bn_apply_backward(dout, a_last, ad, bn_l, ds[1], 2, g8=(g8a, g8b))
                dA8, dAd8 = _use8(q, g8a), _use8(q, g8b)
            else:
                dA, dAd = bn_act_backward(dout, a_last, ad, out, bn_l, ds[1], 2, True)
                dAd8 = None
            dconv = ds[0]
            # a stride-2 1x1 downsample reaches only the even pixels: write those, no memset of the
            # rest (conv1's dgrad below accumulates with old_sub2 = zeros at the odd ones)
            sparse = dconv.stride == 2 and dconv.kh == 1 and dconv.kw == 1 and dconv.padding == 0
            dX = igemm_dgrad(dAd, dconv.wt_bf16, (H, W), dconv.stride, dconv.padding, dconv.kh, dconv.kw,
                             fp8=_dg8(dAd8, dconv), sparse=sparse)
            conv_wgrad(dconv, dAd, x)
        elif premasked and ctx.gram and fuse:
            # dx3 kept as (g, A, B, c): no apply pass (ops/bn_gram.py); when the next block's dgrad ran without x3,
            # sum(g xhat3) comes from T = g^T h2 (formed here, reused by the weight gradient)
            T = gram_T(dout, outs[-1], out=_gws(block, 0)) if getattr(block, "_bnb_nox", False) else None
            dA = gram_coef(bn_l, dout, T=T, w3=conv_l.w_bf16 if T is not None else None, hs=ctx.h2sum)
            dX = dout
        elif premasked:
            g8a = q.grad_out(a_last, bn_l) if (q is not None and fp8_dgrad_ok(conv_l)) else None
            dA, _ = bn_apply_backward(dout, a_last, None, bn_l, None, 1, g8=(g8a, None))
            dA8 = _use8(q, g8a)
            dX = dout  # masked upstream gradient = identity-branch gradient; conv1 dgrad adds into it
        else:
            dA, dX = bn_act_backward(dout, a_last, x, out, bn_l, None, 1, True)  # dX = masked dout
        streams.flush_deferred()  # the next block's conv1 wgrad, after this memory-bound BN pass
        block._last_bn = None
        block._bnb_done = False
        block._bnb_nox = False
        xbn = ctx.xbn  # xbn[i]: conv i's input is BN(acts[i - 1]) + ReLU applied on its operand path
        g_read = None  # side-stream event after the Gram wgrad's last read of dout (= dX)
        for i in range(n - 1, -1, -1):
            conv = pairs[i][0]
            h_in = inputs[i]
            if i > 0:
                bn_prev = pairs[i - 1][1]
                fz = BNBwdFuse(acts[i - 1], bn_prev) if fuse else None
                if isinstance(dA, GramBN):
                    dH = gram_dgrad(dA, conv, h_in, fz, Q=_gws(block, 3))
                    g_read = gram_wgrad(conv, dA, h_in, ctx.h2sum, G=_gws(block, 1), P=ctx.gram_P,
                                        bn=bn_l, T_out=_gws(block, 0), P_out=_gws(block, 4))  # issued now: it reads dout, which conv1's dgrad
                else:                                    # accumulates into below
                    dH = igemm_dgrad(dA, conv.wt_bf16, (acts[i - 1].shape[1], acts[i - 1].shape[2]), conv.stride,
                                     conv.padding, conv.kh, conv.kw, bnb=fz, fp8=_dg8(dA8, conv))
                if h_in is None:  # xfuse: the weight gradient applies the BN on its operand staging
                    h_in = (acts[i - 1], xbn[i])
                dA_w = dA
                if fz is not None:
                    g8a = q.grad_out(acts[i - 1], bn_prev) if (q is not None and fp8_dgrad_ok(pairs[i - 1][0])) else None
                    dA, _ = bn_apply_backward(dH, acts[i - 1], None, bn_prev, None, 0, g8=(g8a, None))
                    dA8 = _use8(q, g8a)
                else:
                    dA, _ = bn_act_backward(dH, acts[i - 1], None, None, bn_prev, None, 0, True)
                    dA8 = None
                if not isinstance(dA_w, GramBN):
                    # issued after the BN-backward pass: the side-stream weight gradient then runs
                    # beside the next (compute-bound) dgrad instead of the memory-bound BN pass
                    _wgrad(conv, dA_w, h_in)
            else:
                prev = getattr(block, "_prev_block", None)
                fz = None
                nox = False
                if fuse and prev is not None and prev._last_bn is not None:
                    pa, pad_, pym = prev._last_bn
                    pbn = prev.convs_bns()[-1][1]
                    pds = prev.downsample
                    # the previous block's bn3 backward takes the Gram form: sum(g xhat3) from g^T h2, x3 not read
                    nox = _GRAM_NOX and getattr(prev, "_gram", False) and pym is not None
                    fz = BNBwdFuse(None if nox else pa, pbn, y=pym, x2=pad_,
                                   bn2=pds[1] if pds is not None else None)
                if g_read is not None:
                    torch.cuda.current_stream().wait_event(g_read)
                igemm_dgrad(dA, conv.wt_bf16, (H, W), conv.stride, conv.padding, conv.kh, conv.kw, out=dX,
                            accumulate=True, bnb=fz, fp8=_dg8(dA8, conv), old_sub2=(ds is not None and sparse))
                # issued by the previous block's backward after its BN pass
                streams.defer(lambda c=conv, g=dA, h=h_in: conv_wgrad(c, g, h))
                if fz is not None:
                    prev._bnb_done = True
                    prev._bnb_nox = nox
        return dX, None
