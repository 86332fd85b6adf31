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
