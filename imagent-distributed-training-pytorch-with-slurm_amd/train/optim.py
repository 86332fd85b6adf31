"""Optimizers over the flat parameter arena.

Reference: ``SGD(model.parameters(), lr, momentum=0.9, weight_decay=1e-4)``
(``imagenet.py:325``) plus the commented-out alternatives Adagrad, RMSprop,
Adadelta, Adam, ASGD, custom Nadam(schedule_decay=4e-3) and custom FR
(``imagenet.py:326-340``; the ``custom_optimizers`` module is missing from the
reference, quirk Q5).

* :class:`FlatSGD` - torch.optim.SGD math ([torch] optim/sgd.py:343-380,
  incl. the first-step ``buf = grad`` rule, dampening and nesterov) as ONE
  fused HIP launch over the whole arena that also rewrites the bf16 compute
  shadow; on CPU the same math in flat torch ops.
* every other optimizer is the stock ``torch.optim`` class over the arena
  views (updates land in the arena) followed by a shadow refresh.
  ``nadam`` maps Keras' ``schedule_decay`` to torch's ``momentum_decay`` (the
  same psi in mu_t = beta1 * (1 - 0.5 * 0.96 ** (t * psi))).
* :class:`FlatLARS` - LARS for the large-batch (8192) configuration.
* ``fr`` is deliberately absent: the reference never defines it.
"""

from __future__ import annotations

from typing import Callable, Dict, List, Optional

import torch

from ..models.arena import ParamArena


class FlatSGD:
    def __init__(self, arena: ParamArena, lr: float, momentum: float = 0.9, dampening: float = 0.0,
                 weight_decay: float = 1e-4, nesterov: bool = False, native: Optional[bool] = None,
                 after_step: Optional[Callable[[], None]] = None):
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        self.arena = arena
        self.native = arena.P.is_cuda if native is None else native
        self.after_step = after_step
        self.param_groups = [dict(lr=lr, momentum=momentum, dampening=dampening,
                                  weight_decay=weight_decay, nesterov=nesterov)]
        self.buf: Optional[torch.Tensor] = None
        self.steps = 0
        self.grad_scale = 1.0

    @property
    def lr(self) -> float:
        return self.param_groups[0]["lr"]

    def zero_grad(self, set_to_none: bool = False) -> None:
        self.arena.zero_grad()

    def flats(self) -> List[torch.Tensor]:
        return [self.buf] if self.buf is not None else []

    def set_flats(self, flats: List[torch.Tensor]) -> None:
        if flats:
            self.buf = flats[0]

    @torch.no_grad()
    def step(self) -> None:
        g = self.param_groups[0]
        lr, mu, damp, wd, nest = g["lr"], g["momentum"], g["dampening"], g["weight_decay"], g["nesterov"]
        ar = self.arena
        first = self.buf is None
        if first and mu != 0:
            self.buf = torch.zeros_like(ar.P)
        if self.native:
            from ..ops.misc import sgd_flat
            sgd_flat(ar.P, ar.G, self.buf, ar.S, lr, mu, damp, wd, nest, first, self.grad_scale)
        else:
            d = ar.G.mul(self.grad_scale) if self.grad_scale != 1.0 else ar.G.clone()
            if wd != 0:
                d.add_(ar.P, alpha=wd)
            if mu != 0:
                if first:
                    self.buf.copy_(d)
                else:
                    self.buf.mul_(mu).add_(d, alpha=1 - damp)
                d = d.add(self.buf, alpha=mu) if nest else self.buf
            ar.P.add_(d, alpha=-lr)
            if ar.S is not None:
                ar.S.copy_(ar.P)
        self.steps += 1
        if self.after_step is not None:
            self.after_step()

    # checkpointing: momentum keyed by parameter name (layout-independent)
    def state_dict(self) -> Dict:
        ar = self.arena
        mom = {}
        if self.buf is not None:
            for i, n in enumerate(ar.names):
                mom[n] = ar.flat_slice(self.buf, i).detach().cpu().clone()
        return {"kind": "sgd", "param_groups": [dict(x) for x in self.param_groups], "steps": self.steps,
                "momentum": mom}

    def load_state_dict(self, sd: Dict) -> None:
        self.param_groups = [dict(x) for x in sd["param_groups"]]
        self.steps = sd.get("steps", 0)
        mom = sd.get("momentum", {})
        ar = self.arena
        if mom:
            self.buf = torch.zeros_like(ar.P)
            for i, n in enumerate(ar.names):
                ar.flat_slice(self.buf, i).copy_(mom[n].to(ar.P.device).reshape(-1))
        else:
            self.buf = None


class FlatLARS(FlatSGD):
    """LARS (You, Gitman, Ginsburg 2017) for large-batch runs (the fp8 8192
    config): per tensor trust = eta * ||w|| / (||g|| + wd * ||w||),
    v = mu * v + lr * trust * (g + wd * w), w -= v. One-dimensional tensors
    (BatchNorm affine, biases) are neither adapted nor decayed. On the GPU it
    is two launches over a per-tensor descriptor table (csrc/kernels/optim.hip);
    on CPU the same math per tensor."""

    def __init__(self, arena: ParamArena, lr: float, momentum: float = 0.9, weight_decay: float = 1e-4,
                 eta: float = 1e-3, native: Optional[bool] = None, after_step: Optional[Callable[[], None]] = None):
        super().__init__(arena, lr, momentum, 0.0, weight_decay, False, native, after_step)
        self.param_groups[0]["eta"] = eta
        self._descs = None

    def _build_descs(self):
        import ctypes as C

        from ..ops import _lib
        ar = self.arena
        T = len(ar.params)
        d = (_lib.LarsDesc * T)()
        for i in range(T):
            o, n = ar.offsets[i], ar.numels[i]
            d[i].p = ar.P[o:o + n].data_ptr()
            d[i].g = ar.G[o:o + n].data_ptr()
            d[i].buf = self.buf[o:o + n].data_ptr()
            d[i].shadow = ar.S[o:o + n].data_ptr() if ar.S is not None else None
            d[i].n = n
            d[i].adapt = 1 if len(ar.shapes[i]) > 1 else 0
        self._descs = torch.frombuffer(bytearray(bytes(memoryview(d))), dtype=torch.uint8).to(ar.P.device)
        self._norms = torch.zeros(2 * T, dtype=torch.float32, device=ar.P.device)
        self._key = (ar.P.data_ptr(), ar.G.data_ptr(), self.buf.data_ptr())
        self._max_n = max(ar.numels)
        del C

    @torch.no_grad()
    def step(self) -> None:
        g = self.param_groups[0]
        lr, mu, wd, eta = g["lr"], g["momentum"], g["weight_decay"], g["eta"]
        ar = self.arena
        first = self.buf is None
        if first:
            self.buf = torch.zeros_like(ar.P)
        if self.native:
            from ..ops import _lib
            if self._descs is None or self._key != (ar.P.data_ptr(), ar.G.data_ptr(), self.buf.data_ptr()):
                self._build_descs()  # (re)built after a bucket re-layout moved the arenas
            _lib.check(_lib.kernels().imk_lars_step(self._descs.data_ptr(), len(ar.params), self._max_n,
                                                    self._norms.data_ptr(), lr, mu, wd, eta, self.grad_scale,
                                                    1 if first else 0, _lib.stream_ptr()), "lars step")
        else:
            for i in range(len(ar.params)):
                w, gr, v = ar.flat_slice(ar.P, i), ar.flat_slice(ar.G, i) * self.grad_scale, \
                    ar.flat_slice(self.buf, i)
                adapt = len(ar.shapes[i]) > 1
                trust, wdt = 1.0, 0.0
                if adapt:
                    wdt = wd
                    wn, gn = w.norm().item(), gr.norm().item()
                    if wn > 0 and gn > 0:
                        trust = eta * wn / (gn + wd * wn)
                d = gr + wdt * w
                if first:
                    v.copy_(lr * trust * d)
                else:
                    v.mul_(mu).add_(d, alpha=lr * trust)
                w.sub_(v)
            if ar.S is not None:
                ar.S.copy_(ar.P)
        self.steps += 1
        if self.after_step is not None:
            self.after_step()

    def state_dict(self) -> Dict:
        sd = super().state_dict()
        sd["kind"] = "lars"
        return sd


class TorchOptimizer:
    """A stock torch.optim optimizer over the arena views + shadow refresh."""

    def __init__(self, arena: ParamArena, opt: torch.optim.Optimizer,
                 after_step: Optional[Callable[[], None]] = None, full_refresh: Optional[Callable] = None):
        self.arena, self.opt = arena, opt
        self.after_step = after_step
        self.full_refresh = full_refresh
        self.steps = 0

    @property
    def param_groups(self):
        return self.opt.param_groups

    def zero_grad(self, set_to_none: bool = False):
        self.arena.zero_grad()

    def flats(self):
        return []

    def set_flats(self, flats):
        pass

    def step(self):
        self.opt.step()
        self.steps += 1
        if self.full_refresh is not None:
            self.full_refresh()

    def state_dict(self):
        return {"kind": "torch", "state": self.opt.state_dict(), "steps": self.steps}

    def load_state_dict(self, sd):
        self.opt.load_state_dict(sd["state"])
        self.steps = sd.get("steps", 0)


def build_optimizer(name: str, arena: ParamArena, lr: float, momentum: float = 0.9,
                    weight_decay: float = 1e-4, nesterov: bool = False,
                    after_step: Optional[Callable[[], None]] = None,
                    full_refresh: Optional[Callable[[], None]] = None, **kw):
    name = name.lower()
    params = arena.params
    if name == "sgd":
        return FlatSGD(arena, lr, momentum, kw.get("dampening", 0.0), weight_decay, nesterov,
                       after_step=after_step)
    if name == "lars":
        return FlatLARS(arena, lr, momentum, weight_decay, eta=kw.get("lars_eta", 1e-3), after_step=after_step)
    if name == "adagrad":
        o = torch.optim.Adagrad(params, lr=lr, lr_decay=0, weight_decay=weight_decay,
                                initial_accumulator_value=0, eps=1e-10)
    elif name == "rmsprop":
        o = torch.optim.RMSprop(params, lr=lr, alpha=0.99, eps=1e-8, weight_decay=weight_decay,
                                momentum=momentum, centered=False)
    elif name == "adadelta":
        o = torch.optim.Adadelta(params, lr=lr, rho=0.9, eps=1e-6, weight_decay=weight_decay)
    elif name == "adam":
        o = torch.optim.Adam(params, lr=lr, betas=(0.9, 0.999), eps=1e-8, weight_decay=weight_decay)
    elif name == "adamw":
        o = torch.optim.AdamW(params, lr=lr, betas=(0.9, 0.999), eps=1e-8, weight_decay=weight_decay)
    elif name == "asgd":
        o = torch.optim.ASGD(params, lr=lr, lambd=1e-4, alpha=0.75, t0=1e6, weight_decay=weight_decay)
    elif name == "nadam":
        o = torch.optim.NAdam(params, lr=lr, betas=(0.9, 0.999), eps=1e-8, weight_decay=weight_decay,
                              momentum_decay=kw.get("schedule_decay", 4e-3))
    elif name == "fr":
        raise ValueError("optimizer 'FR' comes from the reference's missing custom_optimizers "
                         "module (imagenet.py:36) and is not specified anywhere; not implemented")
    else:
        raise ValueError(f"unknown optimizer {name!r}")
    return TorchOptimizer(arena, o, after_step, full_refresh)
