"""Binding of a ResNet to the MI355X kernel path and its NHWC forward.

``bind_native(model, device, order)`` re-homes the parameters into a
:class:`ParamArena` (fp32 master + grad + bf16 shadow, bucket order), builds
the dgrad weight shadows (batched transpose plan), the stem weight as rows of
7 taps x 4 channels padded to 32 (``[Co][KH][32]``, the row-segment gather of
a 4-channel NHWC input) and one device workspace arena for every BatchNorm
(conv-epilogue statistics slab, backward reduction slab, saved mean/invstd)
that is zeroed with a single memset per training step. Options: BN-backward
fusion into the dgrad epilogue, weight gradients on a second stream, fp8
forward (:class:`Fp8State`).
"""

from __future__ import annotations

import os

import ctypes as C
from typing import List, Optional, Sequence

import torch

from ..ops import _lib
from ..ops.block import BlockFn
from ..ops.bn import BNActFn, bn_eval, running_update
from ..ops.conv import ConvFn, LinearFn, conv_out_size, deterministic, igemm_fwd
from ..ops.misc import AvgPoolFn, BNReluPoolFn, MaxPoolFn, StemFn, TransposePlan, maxpool_eval, stem_fused_ok
from .arena import ParamArena
from .resnet import BasicBlock, BatchNorm2d, BNWork, Bottleneck, Conv2d, Linear, ResNet


def stem_view(t: torch.Tensor, kw: int) -> torch.Tensor:
    """[Co][KH][32] stem weight/grad -> [Co][KH][KW][4] view of its real taps."""
    co, kh, _ = t.shape
    return t[:, :, : kw * 4].view(co, kh, kw, 4)  # splits the unit-stride dim: stays a view


class NativeState:
    def __init__(self, model: ResNet, device: torch.device, order: Optional[Sequence[int]] = None,
                 bnb_fusion: bool = True, fp8: bool = False, wgrad_overlap: bool = True):
        self.device = torch.device(device)
        named = list(model.named_parameters())
        self.arena = ParamArena(named, self.device, order=order, with_shadow=True)
        self.model = model
        # one autograd node per residual block with a hand-scheduled backward
        # (ops/block.py); False = per-op autograd nodes (used to cross-check)
        self.fused_blocks = True
        # BN-backward reductions folded into the producing dgrad's (LDS-staged,
        # coalesced) epilogue (ops/block.py): +11 % img/s at 512 img/GPU
        # deterministic mode: BN-backward reductions by the fixed-order reduce pass, not the dgrad epilogues
        bnb_fusion = bnb_fusion and not deterministic()
        self.bnb_fusion = bnb_fusion
        blocks = list(model.blocks())
        for k, b in enumerate(blocks):
            # a plain reference, NOT a registered submodule (nn.Module.__setattr__ would
            # nest every earlier block into this one's state_dict / parameters())
            object.__setattr__(b, "_prev_block", blocks[k - 1] if k > 0 else None)
            b._fuse_bnb = bnb_fusion
            b._has_next = k + 1 < len(blocks)  # a next block whose conv1 dgrad finishes this block's last BN
            b._last_bn = None
            b._bnb_done = False
        self._bind_shadows()
        self._bind_workspace()
        # weight-gradient kernels on a second HIP stream (ops/streams.py)
        from ..ops import streams
        streams.set_wgrad_overlap(wgrad_overlap)
        self.fp8 = None
        if fp8:
            self.fp8 = Fp8State(self)
            for b in blocks:
                b._q8 = self.fp8
            self._fp8_outputs()

    def _fp8_outputs(self) -> None:
        """Which block outputs need an e4m3 copy: those whose next block reads fp8 in its conv1 or downsample
        conv (``ops.block.fp8_fwd_ok``); the stem pool's likewise for the first block."""
        from ..ops.block import fp8_fwd_ok
        blocks = list(self.model.blocks())

        def reads8(b):
            return fp8_fwd_ok(b.conv1) or (b.downsample is not None and fp8_fwd_ok(b.downsample[0]))
        for k, b in enumerate(blocks):
            b._q8_out = k + 1 < len(blocks) and reads8(blocks[k + 1])
        self._q8_pool = bool(blocks) and reads8(blocks[0])

    # ------------------------------------------------------------ shadows
    def _bind_shadows(self):
        m, ar = self.model, self.arena
        dev = self.device
        st_items = []
        t_numel = 0
        convs: List[Conv2d] = m.convs()
        for c in convs:
            sh = ar.shadow(c.weight).view(c.out_channels, c.kh, c.kw, c.in_channels)
            c.w_bf16 = sh
            c.grad_pad = None
            if c is not m.conv1:
                t_numel += sh.numel()
        fc: Linear = m.fc
        fc.w_bf16 = ar.shadow(fc.weight).view(fc.out_features, fc.in_features)
        t_numel += fc.w_bf16.numel()
        self.T = torch.empty(t_numel, dtype=torch.bfloat16, device=dev)
        off = 0
        for c in convs:
            if c is m.conv1:
                continue
            n = c.w_bf16.numel()
            c.wt_bf16 = self.T[off:off + n].view(c.in_channels, c.kh, c.kw, c.out_channels)
            st_items.append((c.w_bf16, c.wt_bf16, c.out_channels, c.kh * c.kw, c.in_channels))
            off += n
        n = fc.w_bf16.numel()
        fc.wt_bf16 = self.T[off:off + n].view(fc.in_features, fc.out_features)
        st_items.append((fc.w_bf16, fc.wt_bf16, fc.out_features, 1, fc.in_features))
        self.tplan = TransposePlan(st_items, dev)
        # stem: input channels 3 -> 4, kernel row = 7 taps x 4 ch padded to 32
        s = m.conv1
        s.stem = True
        s.w_pad = torch.zeros((s.out_channels, s.kh, 32), dtype=torch.bfloat16, device=dev)
        s.grad_pad = torch.zeros((s.out_channels, s.kh, 32), dtype=torch.float32, device=dev)
        s.w_bf16_real = s.w_bf16
        s.w_bf16 = s.w_pad

    def refresh_shadows(self, full: bool = False) -> None:
        """Bring the bf16 copies in line with the fp32 masters. ``full`` also
        re-casts the masters (after init / checkpoint load); the optimizer
        step already writes ``S`` itself."""
        from ..ops.misc import cast_bf16
        if full:
            cast_bf16(self.arena.P, self.arena.S)
        self.tplan.run()
        s = self.model.conv1
        src = s.w_bf16_real
        if src.is_cuda and src.is_contiguous():
            _lib.check(_lib.kernels().imk_stem_pad(src.data_ptr(), s.w_pad.data_ptr(), s.out_channels, s.kh, s.kw,
                                                   s.in_channels, _lib.stream_ptr()), "stem pad")
        else:
            stem_view(s.w_pad, s.kw)[..., : s.in_channels].copy_(src)
        if getattr(self, "fp8", None) is not None:
            self.fp8.after_step()

    def rebind(self) -> None:
        """After an arena re-layout (bucket rebuild): re-point every shadow."""
        self._aff_dev = None  # the eval-affine table holds raw pointers into the old arena: rebuild it lazily
        self._bind_shadows()
        if self.fp8 is not None:
            self.fp8 = Fp8State(self)
            for b in self.model.blocks():
                b._q8 = self.fp8
            self._fp8_outputs()
        self.refresh_shadows(full=True)

    # ---------------------------------------------------------- workspace
    def _bind_workspace(self):
        bns: List[BatchNorm2d] = self.model.batchnorms()
        sizes = [bn.num_features for bn in bns]
        S = _lib.STAT_SLOTS
        nbw = _lib.kernels().imk_bn_bwd_scratch_floats(1)
        per = [(2 * S + nbw) * c for c in sizes]        # stats slab + bwd slab/scratch (zeroed)
        # the Gram-form bn3 accumulators per bottleneck (ops/bn_gram.py): T = g^T h2 [4p][p], G = h2^T h2 [p][p],
        # colsum(h2) [p], Q = W3^T diag(B) W3 [p][p], P = W3 Gc [4p][p] -- zeroed with the slabs by the one per-step
        # memset (the kernels that form them accumulate)
        gram = [(b, b.convs_bns()[-1][0]) for b in self.model.blocks() if len(b.convs_bns()) == 3]
        gsz = [2 * c3.out_channels * c3.in_channels + c3.in_channels * (2 * c3.in_channels + 1) for _, c3 in gram]
        self.zero_ws = torch.zeros(sum(per) + sum(gsz), dtype=torch.float32, device=self.device)
        go = sum(per)
        for (b, c3), n in zip(gram, gsz):
            C4, p = c3.out_channels, c3.in_channels
            w = self.zero_ws[go:go + n]
            o1, o2, o3, o4 = C4 * p, C4 * p + p * p, C4 * p + p * p + p, C4 * p + 2 * p * p + p
            b._gram_ws = (w[:o1].view(C4, p), w[o1:o2].view(p, p), w[o2:o3], w[o3:o4].view(p, p),
                          w[o4:o4 + C4 * p].view(C4, p))
            go += n
        self.save_ws = torch.zeros(sum(4 * c for c in sizes), dtype=torch.float32, device=self.device)
        o = so = 0
        descs = (_lib.RunDesc * len(bns))()
        for i, bn in enumerate(bns):
            c = bn.num_features
            slab = self.zero_ws[o:o + 2 * S * c].view(S, 2, c)
            scratch = self.zero_ws[o + 2 * S * c:o + (2 * S + nbw) * c]
            stats = self.save_ws[so:so + 2 * c]
            save = self.save_ws[so + 2 * c:so + 4 * c]
            bn.work = BNWork(slab, stats, save, scratch)
            o += (2 * S + nbw) * c
            so += 4 * c
            d = descs[i]
            d.sums, d.rmean, d.rvar = stats.data_ptr(), bn.running_mean.data_ptr(), bn.running_var.data_ptr()
            d.nbt = bn.num_batches_tracked.data_ptr()
            d.C = c
            d.momentum = bn.momentum
        self._run_descs = descs
        self.bns = bns

    def eval_affines(self) -> None:
        """Every BN's inference [scale; shift] (``bn._eval_aff``, the conv epilogue's IG_AFFINE operand) from the
        current weights / running statistics: one launch over a descriptor table per eval forward."""
        if getattr(self, "_aff_dev", None) is None:
            sizes = [bn.num_features for bn in self.bns]
            self._aff_buf = torch.empty(sum(2 * c for c in sizes), dtype=torch.float32, device=self.device)
            descs = (_lib.AffDesc * len(self.bns))()
            o = 0
            for d, bn in zip(descs, self.bns):
                c = bn.num_features
                bn._eval_aff = self._aff_buf[o:o + 2 * c].view(2, c)
                d.gamma, d.beta = bn.weight.data_ptr(), bn.bias.data_ptr()
                d.rmean, d.rvar = bn.running_mean.data_ptr(), bn.running_var.data_ptr()
                d.out, d.C, d.eps = bn._eval_aff.data_ptr(), c, bn.eps
                o += 2 * c
            raw = bytes(memoryview(descs))
            self._aff_dev = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(self.device)
        _lib.check(_lib.kernels().imk_bn_eval_affine(self._aff_dev.data_ptr(), len(self.bns), _lib.stream_ptr()),
                   "bn eval affine")

    def running_update(self, rows: List[int]) -> None:
        """After a training forward: update every BN's running stats in one launch."""
        key = tuple(rows)
        if getattr(self, "_run_key", None) != key:
            for d, r in zip(self._run_descs, rows):
                d.inv_cnt = 1.0 / r
                d.unbias = r / max(1, r - 1)
            raw = bytes(memoryview(self._run_descs))
            self._run_dev = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(self.device)
            self._run_key = key
        running_update(self._run_dev, len(self.bns))


class Fp8State:
    """fp8 (``--dtype fp8``): e4m3 shadows of the non-stem conv weights (exact per-step scales), e4m3
    copies of the activations an fp8 forward conv reads and e5m2 copies of the gradients an fp8 dgrad reads
    (delayed per-tensor scales, written by the producing BN / pool pass). Which convs run fp8 is per shape
    (``ops.block.fp8_fwd_ok`` / ``fp8_dgrad_ok``: where the 1-byte v3 loop measured faster); weight
    gradients and everything else stay bf16."""

    def __init__(self, st: "NativeState", backward: bool = True):
        from ..ops.fp8 import E5M2_MAX, ActScales, WeightQuantizer
        m = st.model
        convs = [c for c in m.convs() if c is not m.conv1]
        self.wq = WeightQuantizer([c.weight for c in convs], st.device, transposed=backward)
        for c, v, vt, i in zip(convs, self.wq.views, self.wq.views_t, range(len(convs))):
            c.w8 = v.view(c.out_channels, c.kh, c.kw, c.in_channels)
            c.wt8 = vt  # [Ci][KH][KW][Co] e4m3 (fp8 dgrad) or None
            c.w8_exp = self.wq.exp[i:i + 1]
        bns = m.batchnorms()
        self.slot = {id(bn): i for i, bn in enumerate(bns)}
        self.pool_slot = len(bns)
        self.act = ActScales(len(bns) + 1, st.device)
        # e5m2 copies of the BN-backward outputs (the dgrad inputs), delayed
        # scaling; the first step only observes (bf16 dgrad) so the initial
        # exponent never has to guess the gradient magnitude
        self.backward = backward
        self.grad = ActScales(len(bns), st.device, fmt_max=E5M2_MAX) if backward else None
        self.grad_ready = False
        self.map = {}
        self.active = False
        self.wq.run()

    def after_step(self) -> None:
        """Masters changed: re-quantise weights; this step's amax -> next exponents."""
        self.wq.run()
        self.act.step()
        if self.grad is not None:
            self.grad.step()
            self.grad_ready = True

    def grad_out(self, like: torch.Tensor, bn):
        """(e5m2 buffer, exponent view, amax row) for a BN-backward output, or None."""
        if self.grad is None or like.shape[-1] % 16 or 256 % (like.shape[-1] // 8):
            return None
        i = self.slot[id(bn)]
        return (torch.empty(like.shape, dtype=torch.uint8, device=like.device), self.grad.exp[i:i + 1],
                self.grad.amax[i])

    def begin_forward(self) -> None:
        self.map.clear()
        self.active = True

    def end_forward(self) -> None:
        self.map.clear()
        self.active = False

    def out_for(self, like: torch.Tensor, slot: int):
        """(y8 buffer, exponent view, amax view) for a BN / pool output of this shape."""
        if like.shape[-1] % 16 or 256 % (like.shape[-1] // 8):
            return None
        return (torch.empty(like.shape, dtype=torch.uint8, device=like.device), self.act.exp[slot:slot + 1],
                self.act.amax[slot])

    def register(self, y: torch.Tensor, q8) -> None:
        if q8 is not None:
            self.map[y.data_ptr()] = (q8[0], q8[1])

    def lookup(self, y: torch.Tensor):
        return self.map.get(y.data_ptr())


def bind_native(model: ResNet, device, order: Optional[Sequence[int]] = None,
                bnb_fusion: bool = True, fp8: bool = False, wgrad_overlap: bool = True) -> NativeState:
    model.to(device)
    st = NativeState(model, device, order, bnb_fusion=bnb_fusion, fp8=fp8, wgrad_overlap=wgrad_overlap)
    model.native = st
    model.backend = "hip"
    st.refresh_shadows(full=True)
    return st


# --------------------------------------------------------------------------
# forward
# --------------------------------------------------------------------------

def _conv(x, conv: Conv2d, bn: Optional[BatchNorm2d], train: bool):
    if train:
        return ConvFn.apply(x, conv.weight, conv, bn.work if bn is not None else None)
    return igemm_fwd(x, conv.w_bf16, conv.stride, conv.padding, conv.kh, conv.kw,
                     stem=getattr(conv, "stem", False))


# the stem's BN+ReLU and maxpool as one autograd node (ops.misc.BNReluPoolFn: BN applied inside the pool forward,
# the BN-backward reductions carried by the pool backward); the deterministic mode keeps separate nodes
_FUSED_STEM = True


def _bn(x, bn, relu, train, x2=None, bn2=None, mode=0):
    if train:
        return BNActFn.apply(x, x2, bn, bn2, mode, relu)
    return bn_eval(x, bn, relu, x2=x2, bn2=bn2, mode=mode)


def forward_hip(model: ResNet, x: torch.Tensor) -> torch.Tensor:
    """x: NHWC bf16 [N, H, W, 4] (normalised, channel 3 zero) -> fp32 logits."""
    st: NativeState = model.native
    if x.dtype != torch.bfloat16 or x.dim() != 4 or x.shape[-1] != ResNet.STEM_CPAD:
        raise ValueError(f"hip backend expects NHWC bf16 [N,H,W,{ResNet.STEM_CPAD}], got "
                         f"{tuple(x.shape)} {x.dtype}")
    train = model.training and torch.is_grad_enabled()
    if train:
        _lib.zero_(st.zero_ws)
    q = st.fp8 if (train and st.fused_blocks) else None
    if q is not None:
        q.begin_forward()
    if not train:
        return _forward_eval(model, x)
    rows = []
    if _FUSED_STEM and not deterministic() and stem_fused_ok(x, model.conv1):
        # conv + BN + ReLU + maxpool as one node: the stem BN's backward apply rides in the stem weight gradient
        # (ops.misc.StemFn; same-box in-step A/B 17,061 / 17,085 vs 16,809 / 16,873 img/s at 2048 img/GPU)
        c1 = model.conv1
        rows.append(x.shape[0] * conv_out_size(x.shape[1], c1.kh, c1.stride, c1.padding) *
                    conv_out_size(x.shape[2], c1.kw, c1.stride, c1.padding))
        y = StemFn.apply(x, c1.weight, c1, model.bn1, 3, 2, 1)
    elif _FUSED_STEM and not deterministic():  # BN+ReLU+maxpool, backward fused (ops.misc.BNReluPoolFn)
        y = _conv(x, model.conv1, model.bn1, train)
        rows.append(y.numel() // y.shape[-1])
        y = BNReluPoolFn.apply(y, model.bn1, 3, 2, 1)
    else:
        y = _conv(x, model.conv1, model.bn1, train)
        rows.append(y.numel() // y.shape[-1])
        y = _bn(y, model.bn1, True, train)
        y = MaxPoolFn.apply(y, 3, 2, 1)
    if q is not None and getattr(st, "_q8_pool", True):
        q8 = q.out_for(y, q.pool_slot)
        if q8 is not None:
            from ..ops.fp8 import quant_act
            quant_act(y.detach(), q8[1], q8[2], out=q8[0])
            q.register(y, q8)
    for b in model.blocks():
        if train and st.fused_blocks:
            y = BlockFn.apply(y, b)
            rows.extend(b._bn_rows)
            continue
        idt = y
        pairs = b.convs_bns()
        out = y
        for conv, bn, relu in pairs[:-1]:
            a = _conv(out, conv, bn, train)
            rows.append(a.numel() // a.shape[-1])
            out = _bn(a, bn, True, train)
        conv, bn, _ = pairs[-1]
        a = _conv(out, conv, bn, train)
        rows.append(a.numel() // a.shape[-1])
        if b.downsample is not None:
            dconv, dbn = b.downsample[0], b.downsample[1]
            ad = _conv(idt, dconv, dbn, train)
            rows.append(ad.numel() // ad.shape[-1])
            y = _bn(a, bn, True, train, x2=ad, bn2=dbn, mode=2)
        else:
            y = _bn(a, bn, True, train, x2=idt, mode=1)
    if q is not None:
        q.end_forward()
    pooled = AvgPoolFn.apply(y) if train else _avg_eval(y)
    if train:
        logits = LinearFn.apply(pooled, model.fc.weight, model.fc)
        st.running_update(_rows_in_bn_order(model, rows))
    else:
        fc = model.fc
        B = pooled.shape[0]
        logits = igemm_fwd(pooled.view(B, 1, 1, -1), fc.w_bf16.view(fc.out_features, 1, 1, -1), 1, 0, 1,
                           1, bias=fc.bias, out_f32=True).view(B, -1)
    return logits


def _affine(bn: BatchNorm2d) -> torch.Tensor:
    """Inference BN as a per-channel [scale; shift] for the conv epilogue (IG_AFFINE)."""
    with torch.no_grad():
        sc = bn.weight * torch.rsqrt(bn.running_var + bn.eps)
        return torch.stack([sc, bn.bias - bn.running_mean * sc]).float().contiguous()


def _forward_eval(model: ResNet, x: torch.Tensor) -> torch.Tensor:
    """Inference: every BatchNorm (+ReLU, +residual) folded into the epilogue
    of the conv that feeds it -- one pass per conv, no BN kernels.
    The block's last conv accumulates onto the shortcut (identity copy or the
    downsample conv's folded output) and applies the ReLU after the sum."""
    st = getattr(model, "native", None)
    st = st if isinstance(st, NativeState) else None
    if st is not None:
        st.eval_affines()  # bn._eval_aff for every BN, one launch

    def conv(h, c, bn, relu, out=None, accumulate=False):
        aff = bn._eval_aff if st is not None else _affine(bn)
        return igemm_fwd(h, c.w_bf16, c.stride, c.padding, c.kh, c.kw, stem=getattr(c, "stem", False),
                         affine=aff, relu=relu, out=out, accumulate=accumulate)

    y = conv(x, model.conv1, model.bn1, True)
    y = maxpool_eval(y, 3, 2, 1)
    for b in model.blocks():
        pairs = b.convs_bns()
        h = y
        for c, bn, _ in pairs[:-1]:
            h = conv(h, c, bn, True)
        c, bn, _ = pairs[-1]
        # the block's last conv accumulates onto the shortcut: the downsample conv's output, or the block
        # input itself, in place (no later reader: every consumer of y in this block has run)
        short = conv(y, b.downsample[0], b.downsample[1], False) if b.downsample is not None else y
        y = conv(h, c, bn, True, out=short, accumulate=True)
    pooled = _avg_eval(y)
    fc = model.fc
    B = pooled.shape[0]
    return igemm_fwd(pooled.view(B, 1, 1, -1), fc.w_bf16.view(fc.out_features, 1, 1, -1), 1, 0, 1, 1,
                     bias=fc.bias, out_f32=True).view(B, -1)


def _avg_eval(y):
    from ..ops.misc import _lib as L
    N, H, W, Cc = y.shape
    out = torch.empty((N, Cc), device=y.device, dtype=y.dtype)
    L.check(L.kernels().imk_avgpool_fwd(y.data_ptr(), out.data_ptr(), N, H * W, Cc, L.stream_ptr()),
            "avgpool")
    return out


def _rows_in_bn_order(model: ResNet, rows_fwd: List[int]) -> List[int]:
    """Map the per-conv row counts (forward order) onto model.batchnorms() order."""
    # forward order: stem, then per block conv1..convK, [downsample]; batchnorms()
    # (module order) lists: bn1, then per block bn1..bnK, [downsample.1] -> identical.
    return rows_fwd
