"""Learning-rate schedules.

Reference: ``lr = initial_lr * 0.1 ** (epoch // 30)`` written into every
param group once per epoch (``adjust_learning_rate``, ``imagenet.py:154-162``;
called at ``imagenet.py:378``). That is :func:`step_lr` with the defaults.

Additions for large global batches (the 8192-image fp8 config; quirk Q9: the
reference uses LR 0.1 at batch 2048 with no warmup): linear LR scaling with the
global batch and a per-iteration linear warmup, plus cosine decay.
"""

from __future__ import annotations

import math


def step_lr(initial_lr: float, epoch: int, step: int = 30, gamma: float = 0.1) -> float:
    return initial_lr * (gamma ** (epoch // step))


def adjust_learning_rate(initial_lr: float, optimizer, epoch: int, step: int = 30,
                         gamma: float = 0.1) -> float:
    """Reference-compatible: sets and returns the epoch's LR (imagenet.py:154)."""
    lr = step_lr(initial_lr, epoch, step, gamma)
    for g in optimizer.param_groups:
        g["lr"] = lr
    return lr


class Schedule:
    """Per-iteration LR: warmup -> {step | cosine} decay, optional linear scaling."""

    def __init__(self, base_lr: float, epochs: int, iters_per_epoch: int, kind: str = "step",
                 step: int = 30, gamma: float = 0.1, warmup_epochs: float = 0.0,
                 scale_batch: int = 0, ref_batch: int = 256):
        self.base = base_lr * (scale_batch / ref_batch if scale_batch else 1.0)
        self.epochs, self.ipe = epochs, max(1, iters_per_epoch)
        self.kind, self.step_size, self.gamma = kind, step, gamma
        self.warmup = warmup_epochs

    def __call__(self, epoch: int, it: int = 0) -> float:
        t = epoch + it / self.ipe
        if self.warmup > 0 and t < self.warmup:
            return self.base * (t + 1.0 / self.ipe) / self.warmup
        if self.kind == "cosine":
            frac = (t - self.warmup) / max(1e-9, self.epochs - self.warmup)
            return 0.5 * self.base * (1 + math.cos(math.pi * min(1.0, frac)))
        return step_lr(self.base, epoch, self.step_size, self.gamma)

    def apply(self, optimizer, epoch: int, it: int = 0) -> float:
        lr = self(epoch, it)
        for g in optimizer.param_groups:
            g["lr"] = lr
        return lr
