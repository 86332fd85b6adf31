"""ResNet on the fp32 HIP kernels (``--dtype fp32 --kernels hip``): the reference's own precision.

The reference trains torchvision's resnet18 in fp32 at 448x448 (``/root/reference/imagenet.py:281,
312``). ``bind_native_f32`` re-homes the parameters into a :class:`ParamArena` (fp32 masters and
gradients in bucket order, no bf16 shadows) and routes ``model.forward`` through
:func:`forward_hip_f32`: NHWC fp32 activations, convolutions on the exact-f32 MFMA, BatchNorm with
deterministic statistics, ReLU / residual add fused into the BN apply, maxpool / avgpool / fc on
own kernels (``ops/f32.py``, ``csrc/kernels/f32.hip``). Training runs each residual block as one autograd
node (``BlockF32Fn``: BatchNorm statistics summed in the conv epilogues, the residual gradient accumulated in
conv1's dgrad epilogue, weight gradients on the side stream); the stem and fc are per-op nodes. Weight
gradients go straight into the arena and notify the bucketed reducer, so the data-parallel path
(``parallel/ddp.py``) is the same as for bf16.
"""

from __future__ import annotations

from typing import Optional, Sequence

import torch

from ..ops.f32 import (AvgPoolF32Fn, BlockF32Fn, BNF32Fn, ConvF32Fn, F32Workspace, LinearF32Fn, MaxPoolF32Fn,
                       avgpool_f32, bn_eval_f32, conv_f32, maxpool_f32, _weight_nhwc)
from .arena import ParamArena
from .resnet import ResNet


class NativeF32State:
    def __init__(self, model: ResNet, device, order: Optional[Sequence[int]] = None, wgrad_overlap: bool = True):
        self.device = torch.device(device)
        # weight gradients on the second HIP stream (ops/streams.py), as on the bf16 path
        from ..ops import streams
        streams.set_wgrad_overlap(wgrad_overlap)
        self.model = model
        self.arena = ParamArena(list(model.named_parameters()), self.device, order=order, with_shadow=False)
        cmax = max(bn.num_features for bn in model.batchnorms())
        self.ws = F32Workspace(self.device, cmax)
        # one autograd node per residual block (ops/f32.py BlockF32Fn); False: per-op nodes (cross-check)
        self.fused_blocks = True

    def refresh_shadows(self, full: bool = False) -> None:
        """No low-precision shadows on the fp32 path (optimizer hook no-op)."""

    def rebind(self) -> None:
        """After an arena re-layout: the parameters are views of the new arena; nothing else to do."""


def bind_native_f32(model: ResNet, device, order: Optional[Sequence[int]] = None) -> NativeF32State:
    model.to(device)
    st = NativeF32State(model, device, order)
    model.native = st
    model.backend = "hip_f32"
    return st


def _bn(x, bn, relu, ws, train, res=None):
    if train:
        return BNF32Fn.apply(x, res, bn, relu, ws)
    return bn_eval_f32(x, bn, res, relu)


def _conv(x, conv, train, bn=None):
    """``bn``: the BatchNorm right after this conv -- its training statistics are summed in the conv's
    epilogue (one pass less over the activation; the fixed-order partial passes in deterministic mode)."""
    if train:
        from ..ops.conv import deterministic
        return ConvF32Fn.apply(x, conv.weight, conv, None if deterministic() else bn)
    return conv_f32(x, _weight_nhwc(conv, x.shape[-1]), conv.stride, conv.padding, conv.kh, conv.kw)


def forward_hip_f32(model: ResNet, x: torch.Tensor) -> torch.Tensor:
    """x: NHWC fp32 [N, H, W, 4] (normalised, channel 3 zero) -> fp32 logits."""
    st: NativeF32State = model.native
    if x.dtype != torch.float32 or x.dim() != 4 or x.shape[-1] != ResNet.STEM_CPAD:
        raise ValueError(f"hip_f32 backend expects NHWC fp32 [N,H,W,{ResNet.STEM_CPAD}], got "
                         f"{tuple(x.shape)} {x.dtype}")
    train = model.training and torch.is_grad_enabled()
    ws = st.ws
    y = _bn(_conv(x, model.conv1, train, model.bn1), model.bn1, True, ws, train)
    y = MaxPoolF32Fn.apply(y, 3, 2, 1) if train else maxpool_f32(y, 3, 2, 1)[0]
    for b in model.blocks():
        if train and st.fused_blocks:  # one autograd node per block (ops/f32.py BlockF32Fn)
            y = BlockF32Fn.apply(y, b, ws)
            continue
        h = y
        pairs = b.convs_bns()
        for conv, bn, _ in pairs[:-1]:
            h = _bn(_conv(h, conv, train, bn), bn, True, ws, train)
        conv, bn, _ = pairs[-1]
        a = _conv(h, conv, train, bn)
        if b.downsample is not None:
            idt = _bn(_conv(y, b.downsample[0], train, b.downsample[1]), b.downsample[1], False, ws, train)
        else:
            idt = y
        y = _bn(a, bn, True, ws, train, res=idt)
    pooled = AvgPoolF32Fn.apply(y) if train else avgpool_f32(y)
    fc = model.fc
    if train:
        return LinearF32Fn.apply(pooled, fc.weight, fc.bias, fc)
    B = pooled.shape[0]
    w = fc.weight.detach()
    return conv_f32(pooled.view(B, 1, 1, -1), w.view(w.shape[0], 1, 1, -1), 1, 0, 1, 1,
                    bias=fc.bias.detach()).view(B, -1)
