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
* skip the ReLU-output read in BN backward (mask recomputed from x).

It also removes ~6 autograd nodes and their Python dispatch per block.
"""

from __future__ import annotations

import torch

from .bn import bn_act_backward, bn_act_forward
from .conv import conv_wgrad, igemm_dgrad, igemm_fwd


def _fwd(conv, h, bn):
    return igemm_fwd(h, conv.w_bf16, conv.stride, conv.padding, conv.kh, conv.kw,
                     stats=bn.work.slab, stem=getattr(conv, "stem", False))


class BlockFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, block):
        pairs = block.convs_bns()
        saved = [x]
        h = x
        for conv, bn, _ in pairs[:-1]:
            a = _fwd(conv, h, bn)
            h = bn_act_forward(a, None, bn, None, 0, True)
            saved += [a, h]
        conv, bn, _ = pairs[-1]
        a = _fwd(conv, h, bn)
        ds = block.downsample
        if ds is not None:
            ad = _fwd(ds[0], x, ds[1])
            out = bn_act_forward(a, ad, bn, ds[1], 2, True)
        else:
            ad = None
            out = bn_act_forward(a, x, bn, None, 1, True)
        saved += [a, ad, out]
        # rows seen by each BN (module order: bn1..bnK, downsample.1) for the running-stat update
        rows = [t.numel() // t.shape[-1] for t in saved[1:-3:2]] + [a.numel() // a.shape[-1]]
        if ad is not None:
            rows.append(ad.numel() // ad.shape[-1])
        block._bn_rows = rows
        ctx.block = block
        ctx.save_for_backward(*saved)
        return out

    @staticmethod
    def backward(ctx, dout):
        block = ctx.block
        pairs = block.convs_bns()
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
        if ds is not None:
            dA, dAd = bn_act_backward(dout, a_last, ad, out, bn_l, ds[1], 2, True)
            dconv = ds[0]
            dX = igemm_dgrad(dAd, dconv.wt_bf16, (H, W), dconv.stride, dconv.padding, dconv.kh, dconv.kw)
            conv_wgrad(dconv, dAd, x)
        else:
            dA, dX = bn_act_backward(dout, a_last, x, out, bn_l, None, 1, True)  # dX = masked dout
        for i in range(n - 1, -1, -1):
            conv = pairs[i][0]
            h_in = inputs[i]
            if i > 0:
                dH = igemm_dgrad(dA, conv.wt_bf16, (h_in.shape[1], h_in.shape[2]), conv.stride, conv.padding,
                                 conv.kh, conv.kw)
                conv_wgrad(conv, dA, h_in)
                dA, _ = bn_act_backward(dH, acts[i - 1], None, None, pairs[i - 1][1], None, 0, True)
            else:
                igemm_dgrad(dA, conv.wt_bf16, (H, W), conv.stride, conv.padding, conv.kh, conv.kw, out=dX,
                            accumulate=True)
                conv_wgrad(conv, dA, h_in)
        return dX, None
