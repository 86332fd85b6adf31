"""Flat parameter / gradient / shadow arenas.

Every trainable parameter of a model is re-homed into ONE flat fp32 buffer
(``P``) laid out in gradient-bucket order, with its gradient in a parallel
buffer (``G``) and - on the GPU path - its bf16 compute copy in ``S``.
Consequences that shape the MI355X design:

* a DDP bucket is a contiguous slice of ``G``: the RCCL all-reduce runs in
  place, there is no bucket copy-in/copy-out (c10d copies every grad into a
  bucket buffer unless ``gradient_as_bucket_view=True``);
* the optimizer step is ONE elementwise launch over ``P``/``G``/momentum that
  also refreshes ``S`` (no foreach multi-tensor metadata);
* ``zero_grad`` is one memset of ``G``; kernels accumulate (``+=``) into it,
  which makes gradient accumulation free.

Conv weights keep torchvision's logical shape ``[Co, Ci, KH, KW]`` but are
stored channels-last (``[Co][KH][KW][Ci]``), the layout the NHWC implicit-GEMM
kernels consume, so the checkpoint keys/shapes stay torchvision-identical.
"""

from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn as nn

ALIGN = 64  # elements (256 B fp32): keeps every slice 16-B aligned for vector loads


def _align(n: int) -> int:
    return (n + ALIGN - 1) // ALIGN * ALIGN


def _as_layout(flat: torch.Tensor, shape: Tuple[int, ...], channels_last: bool) -> torch.Tensor:
    if channels_last and len(shape) == 4:
        co, ci, kh, kw = shape
        return flat.view(co, kh, kw, ci).permute(0, 3, 1, 2)
    return flat.view(shape)


class ParamArena:
    def __init__(self, named_params: Sequence[Tuple[str, nn.Parameter]], device: torch.device,
                 order: Optional[Sequence[int]] = None, with_shadow: bool = False):
        self.names = [n for n, _ in named_params]
        self.params: List[nn.Parameter] = [p for _, p in named_params]
        self.index: Dict[int, int] = {id(p): i for i, p in enumerate(self.params)}
        self.device = torch.device(device)
        self.with_shadow = with_shadow
        self.shapes = [tuple(p.shape) for p in self.params]
        self.channels_last = [p.dim() == 4 for p in self.params]
        self.numels = [p.numel() for p in self.params]
        self._build(list(order) if order is not None else list(range(len(self.params))))

    # ------------------------------------------------------------------
    def _build(self, order: List[int], old: Optional["ParamArena"] = None) -> None:
        assert sorted(order) == list(range(len(self.params))), "order must be a permutation"
        self.order = order
        self.offsets = [0] * len(self.params)
        off = 0
        for i in order:
            self.offsets[i] = off
            off += _align(self.numels[i])
        self.total = off
        P = torch.zeros(self.total, dtype=torch.float32, device=self.device)
        G = torch.zeros(self.total, dtype=torch.float32, device=self.device)
        S = torch.zeros(self.total, dtype=torch.bfloat16, device=self.device) if self.with_shadow else None
        for i, p in enumerate(self.params):
            v = self.view(P, i)
            v.copy_(p.detach().to(self.device, torch.float32))
            gv = self.view(G, i)
            if p.grad is not None:
                gv.copy_(p.grad.detach())
            p.data = v
            p.grad = gv
        self.P, self.G, self.S = P, G, S

    def view(self, flat: torch.Tensor, i: int) -> torch.Tensor:
        o, n = self.offsets[i], self.numels[i]
        return _as_layout(flat[o:o + n], self.shapes[i], self.channels_last[i])

    def flat_slice(self, flat: torch.Tensor, i: int) -> torch.Tensor:
        o, n = self.offsets[i], self.numels[i]
        return flat[o:o + n]

    def shadow(self, p: nn.Parameter) -> torch.Tensor:
        """bf16 compute copy of ``p`` in its storage layout ([Co][KH][KW][Ci] for convs)."""
        i = self.index[id(p)]
        return self.flat_slice(self.S, i)

    def nbytes_of(self, i: int) -> int:
        return self.numels[i] * 4

    def relayout(self, order: Sequence[int], flats: Sequence[torch.Tensor] = ()) -> List[torch.Tensor]:
        """Rebuild with a new bucket order; ``flats`` (e.g. optimizer momentum
        arenas with the same offsets) are remapped and returned."""
        old_offsets = list(self.offsets)
        old_total = self.total
        saved = [t for t in flats]
        self._build(list(order))
        out = []
        for t in saved:
            assert t.numel() == old_total
            n = torch.zeros(self.total, dtype=t.dtype, device=t.device)
            for i in range(len(self.params)):
                n[self.offsets[i]:self.offsets[i] + self.numels[i]] = \
                    t[old_offsets[i]:old_offsets[i] + self.numels[i]]
            out.append(n)
        return out

    def zero_grad(self) -> None:
        from ..ops import _lib
        _lib.zero_(self.G)

    def bucket_param_order(self) -> List[int]:
        return list(self.order)
