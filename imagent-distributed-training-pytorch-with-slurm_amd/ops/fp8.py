"""fp8 (OCP e4m3) quantisation for the fp8 forward path (csrc/kernels/fp8.hip).

Per-tensor power-of-two scales q = x * 2^-e; the exponents stay on the device
and the conv kernel feeds them to the block-scaled MFMA as E8M0 scales, so
neither quantisation nor dequantisation needs a host round trip.

* :class:`WeightQuantizer` -- exact per-step scaling of every conv weight
  (fp32 master -> e4m3 shadow) in two launches over a descriptor table.
* :class:`ActScales` -- delayed scaling for activations: slot i's tensor is
  quantised with the exponent from the previous step's amax, this step's amax
  is recorded, :meth:`ActScales.step` turns amax into next step's exponents.
"""

from __future__ import annotations

import ctypes as C
from typing import List, Sequence

import torch

from . import _lib

E4M3_MAX = 448.0
E5M2_MAX = 57344.0
AMAX_SLOTS = 32  # fp8.hip / bn.hip: per-tensor amax row, folded by imk_fp8_update_exp


def quant_act(x: torch.Tensor, exp: torch.Tensor, amax: torch.Tensor = None,
              out: torch.Tensor = None) -> torch.Tensor:
    """bf16 tensor -> uint8 e4m3 bytes of x * 2^-exp (exp: device int32 scalar);
    ``amax``: the tensor's [AMAX_SLOTS] row of :class:`ActScales`."""
    if out is None:
        out = torch.empty(x.shape, dtype=torch.uint8, device=x.device)
    _lib.check(_lib.kernels().imk_quant_fp8(x.data_ptr(), out.data_ptr(), x.numel(), exp.data_ptr(),
                                            _lib.ptr(amax), _lib.stream_ptr()), "fp8 quant")
    return out


class ActScales:
    """Device exponents + amax accumulators for ``n`` activation (or gradient) tensors."""

    def __init__(self, n: int, device, margin: int = 0, fmt_max: float = E4M3_MAX, init_exp: int = 0):
        self.n = n
        self.exp = torch.full((n,), init_exp, dtype=torch.int32, device=device)
        self.fmt_max = fmt_max
        self.amax = torch.zeros(n, AMAX_SLOTS, dtype=torch.float32, device=device)  # spread atomics
        self.margin = margin

    def step(self) -> None:
        # the kernel sizes exponents for e4m3 (448); e5m2's 57344 = 448 * 2^7
        extra = 0 if self.fmt_max == E4M3_MAX else -7
        _lib.check(_lib.kernels().imk_fp8_update_exp(self.amax.data_ptr(), self.exp.data_ptr(), self.n,
                                                     self.margin + extra, _lib.stream_ptr()), "fp8 update exp")


class WeightQuantizer:
    """e4m3 shadows of fp32 weights, re-quantised (exact amax) by :meth:`run`."""

    def __init__(self, weights: Sequence[torch.Tensor], device, margin: int = 0, transposed: bool = False):
        """``transposed``: also keep [Ci][KH][KW][Co] copies (``views_t``) of
        4-d conv weights for the fp8 dgrad, same per-tensor exponent."""
        dev = torch.device(device)
        total = sum((w.numel() + 15) // 16 * 16 for w in weights)
        self.q = torch.zeros(total, dtype=torch.uint8, device=dev)
        self.qt = torch.zeros(total, dtype=torch.uint8, device=dev) if transposed else None
        self.views_t: List[torch.Tensor] = []
        self.exp = torch.zeros(len(weights), dtype=torch.int32, device=dev)
        self.amax = torch.zeros(len(weights), dtype=torch.float32, device=dev)
        self.views: List[torch.Tensor] = []
        descs = (_lib.QDesc * len(weights))()
        off = 0
        max_n4 = 1
        for i, w in enumerate(weights):
            assert w.numel() % 4 == 0 and (w.is_contiguous(memory_format=torch.channels_last) or w.is_contiguous())
            v = self.q[off:off + w.numel()]
            self.views.append(v)
            d = descs[i]
            d.src, d.dst, d.n4 = w.data_ptr(), v.data_ptr(), w.numel() // 4
            if self.qt is not None and w.dim() == 4:
                co, ci, kh, kw = w.shape
                vt = self.qt[off:off + w.numel()]
                self.views_t.append(vt.view(ci, kh, kw, co))
                d.dstT, d.T, d.Ci = vt.data_ptr(), kh * kw, ci
            else:
                self.views_t.append(None)
            d.exp = self.exp[i:i + 1].data_ptr()
            d.amax = self.amax[i:i + 1].data_ptr()
            max_n4 = max(max_n4, w.numel() // 4)
            off += (w.numel() + 15) // 16 * 16  # 16-B aligned slots
        self._descs = torch.frombuffer(bytearray(bytes(memoryview(descs))), dtype=torch.uint8).to(dev)
        self._n, self._max_n4, self.margin = len(weights), max_n4, margin

    def run(self) -> None:
        _lib.zero_(self.amax)
        _lib.check(_lib.kernels().imk_quant_fp8_weights(self._descs.data_ptr(), self._n, self._max_n4,
                                                        self.margin, _lib.stream_ptr()), "fp8 weights")
