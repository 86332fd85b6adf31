"""Checkpoints.

Reference (``imagenet.py:387-392``): when ``val_prec1 > best_top1`` and the
process is the master and ``--save-model`` is set, ``torch.save(model.
state_dict(), "imagenet_FR_resnet18.pt")`` - a DDP state dict, so every key is
``module.``-prefixed (122 keys for ResNet-18). No optimizer state, no resume.

Here:
* :func:`save_best` writes exactly that layout (``module.`` + torchvision
  keys, standalone contiguous fp32 tensors even though training keeps
  channels-last masters in a flat arena, plus ``_metadata`` with BN
  ``version: 2``), named ``imagenet_FR_<arch>.pt``;
* :func:`save_state` / :func:`load_state` add a full training state
  (model, optimizer momentum, epoch, best metrics, RNG) for ``--resume``
  (SURVEY §5.3/§5.4); loads use ``weights_only=True``.
"""

from __future__ import annotations

import collections
import os
import random
from typing import Any, Dict, Optional

import numpy as np
import torch
import torch.nn as nn


def reference_state_dict(model: nn.Module, prefix: str = "module.") -> "collections.OrderedDict":
    """torchvision-format state dict (contiguous clones, ``module.`` prefix)."""
    sd = model.state_dict()
    out = collections.OrderedDict()
    for k, v in sd.items():
        out[prefix + k] = v.detach().clone().contiguous(memory_format=torch.contiguous_format).cpu()
    meta = collections.OrderedDict()
    src_meta = getattr(sd, "_metadata", {}) or {}
    for k, v in src_meta.items():
        meta[(prefix[:-1] + "." + k) if k else prefix[:-1]] = dict(v)
    meta[""] = {"version": 1}
    # torchvision BatchNorm2d reports version 2 (num_batches_tracked present)
    from ..models.resnet import BatchNorm2d
    for name, m in model.named_modules():
        if isinstance(m, BatchNorm2d):
            key = prefix + name if name else prefix[:-1]
            meta[key] = {"version": 2}
    out._metadata = meta
    return out


def save_best(model: nn.Module, arch: str, directory: str = ".", name: Optional[str] = None) -> str:
    path = os.path.join(directory, name or f"imagenet_FR_{arch}.pt")
    tmp = path + ".tmp"
    torch.save(reference_state_dict(model), tmp)
    os.replace(tmp, path)
    return path


def load_reference_weights(model: nn.Module, path: str) -> None:
    """Load a (``module.``-prefixed or plain) torchvision-layout state dict."""
    sd = torch.load(path, map_location="cpu", weights_only=True)
    sd = {(k[7:] if k.startswith("module.") else k): v for k, v in sd.items()}
    own = model.state_dict()
    missing = [k for k in own if k not in sd]
    if missing:
        raise KeyError(f"checkpoint lacks {len(missing)} keys, e.g. {missing[:4]}")
    with torch.no_grad():
        for k, t in own.items():
            t.copy_(sd[k].to(t.dtype))


def _rng_state() -> Dict[str, Any]:
    st = {"torch": torch.get_rng_state(), "numpy": torch.from_numpy(
        np.frombuffer(np.random.get_state()[1].tobytes(), dtype=np.uint8).copy()),
        "python": torch.tensor(list(random.getstate()[1]), dtype=torch.int64)}
    if torch.cuda.is_available():
        st["cuda"] = torch.cuda.get_rng_state()
    return st


def save_state(path: str, model: nn.Module, optimizer, epoch: int, best: Dict[str, Any],
               extra: Optional[Dict[str, Any]] = None) -> str:
    state = {
        "model": reference_state_dict(model, prefix=""),
        "optimizer": optimizer.state_dict(),
        "epoch": epoch,
        "best": best,
        "rng": _rng_state(),
        "extra": extra or {},
    }
    tmp = path + ".tmp"
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    torch.save(state, tmp)
    os.replace(tmp, path)
    return path


def load_state(path: str, model: nn.Module, optimizer=None) -> Dict[str, Any]:
    state = torch.load(path, map_location="cpu", weights_only=True)
    own = model.state_dict()
    with torch.no_grad():
        for k, t in own.items():
            t.copy_(state["model"][k].to(t.dtype))
    if optimizer is not None and "optimizer" in state:
        optimizer.load_state_dict(state["optimizer"])
    rng = state.get("rng", {})
    if "torch" in rng:
        torch.set_rng_state(rng["torch"])
    if "cuda" in rng and torch.cuda.is_available():
        torch.cuda.set_rng_state(rng["cuda"])
    return state
