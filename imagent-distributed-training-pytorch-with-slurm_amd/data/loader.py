"""Input pipeline: sharded uint8 batches -> pinned host -> async H2D on a HIP
copy stream -> GPU normalise kernel -> model input.

Replaces the reference's ``DataLoader(..., num_workers=10, sampler=
DistributedSampler, pin_memory=True)`` + ``.cuda(non_blocking=True)`` +
CPU ``ToTensor/Normalize`` (``imagenet.py:119-120, 280-283, 346-359``):

* workers only decode + resize to uint8 (4x fewer bytes than the reference's
  fp32 tensors through shared memory, pinning and PCIe: 38.5 MB instead of
  154 MB per 256-image 224^2 batch);
* the next batch's H2D copy runs on a dedicated copy stream while the
  current step computes; the compute stream waits on an event, never on the
  host;
* normalisation (``(x/255 - mean)/std``), the NHWC channel padding for the
  stem and optional random crop / horizontal flip are one HIP kernel;
* workers are persistent (the reference re-forks 10 workers every epoch).
"""

from __future__ import annotations

from typing import Iterator, Optional, Sequence, Tuple

import torch

from ..parallel.sampler import ShardSampler
from .imagenet import collate_u8

MEAN = (0.5, 0.5, 0.5)   # imagenet.py:283
STD = (0.5, 0.5, 0.5)


class InputTransform:
    """uint8 [B,H,W,3] (on the compute device) -> model input."""

    def __init__(self, backend: str, size: Tuple[int, int], mean=MEAN, std=STD, cpad: int = 8,
                 flip: bool = False, dtype=torch.float32, resize: bool = False):
        self.backend, self.size = backend, tuple(size)
        self.mean, self.std, self.cpad = tuple(mean), tuple(std), cpad
        self.flip = flip
        self.dtype = dtype
        # resize: an image of another size is bilinearly resampled to `size` (records stored smaller than the
        # model input, --record-resize) instead of randomly cropped
        self.resize = resize

    def __call__(self, u8: torch.Tensor) -> torch.Tensor:
        B, H, W, _ = u8.shape
        oh, ow = self.size
        if self.backend in ("hip", "hip_f32"):
            from ..ops.misc import normalize_u8
            if self.backend == "hip_f32":  # fp32 NHWC for the fp32 kernel path
                from ..ops.f32 import normalize_u8_f32 as normalize_u8
            crop = flip = None
            if self.flip:
                flip = torch.randint(0, 2, (B,), dtype=torch.uint8, device=u8.device)
            if self.resize and (H, W) != (oh, ow):
                if self.backend == "hip_f32":
                    raise NotImplementedError("--record-resize: the bf16 input path only")
                from ..ops.misc import resize_normalize_u8
                return resize_normalize_u8(u8, (oh, ow), self.cpad, self.mean, self.std, flip)
            if (H, W) != (oh, ow):
                cy = torch.randint(0, H - oh + 1, (B,), dtype=torch.int32, device=u8.device)
                cx = torch.randint(0, W - ow + 1, (B,), dtype=torch.int32, device=u8.device)
                crop = torch.stack([cy, cx], 1).contiguous()
            return normalize_u8(u8, (oh, ow), self.cpad, self.mean, self.std, crop, flip)
        if self.resize and (H, W) != (oh, ow):
            x = torch.nn.functional.interpolate(u8.permute(0, 3, 1, 2).float(), size=(oh, ow), mode="bilinear",
                                                align_corners=False).to(self.dtype).div_(255.0)
        else:
            x = u8[:, :oh, :ow].permute(0, 3, 1, 2).to(self.dtype).div_(255.0)
        m = torch.tensor(self.mean, dtype=self.dtype, device=u8.device).view(1, 3, 1, 1)
        s = torch.tensor(self.std, dtype=self.dtype, device=u8.device).view(1, 3, 1, 1)
        x = (x - m) / s
        if self.flip:
            f = torch.rand(B, device=u8.device) < 0.5
            x[f] = x[f].flip(3)
        return x.contiguous()


class _IndexBatches(torch.utils.data.Sampler):
    def __init__(self, sampler: ShardSampler, batch_size: int, drop_last: bool):
        self.s, self.b, self.d = sampler, batch_size, drop_last

    def __iter__(self):
        for idx in self.s.batches(self.b, self.d):
            yield idx.tolist()

    def __len__(self):
        return self.s.num_batches(self.b, self.d)


class DeviceLoader:
    """Iterates (model_input, labels) for one epoch of one rank's shard."""

    def __init__(self, dataset, sampler: ShardSampler, batch_size: int, transform: InputTransform,
                 device: torch.device, workers: int = 8, drop_last: bool = False,
                 prefetch_factor: int = 4):
        self.dataset, self.sampler, self.batch = dataset, sampler, batch_size
        self.transform, self.device = transform, torch.device(device)
        pin = self.device.type == "cuda"
        kw = dict(num_workers=workers, pin_memory=pin, collate_fn=collate_u8)
        if workers > 0:
            kw.update(persistent_workers=True, prefetch_factor=prefetch_factor)
        self.dl = torch.utils.data.DataLoader(dataset, batch_sampler=_IndexBatches(sampler, batch_size, drop_last),
                                              **kw)
        self.copy_stream = torch.cuda.Stream(self.device) if pin else None

    def __len__(self):
        return len(self.dl)

    def __iter__(self) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        it = iter(self.dl)
        if self.copy_stream is None:
            for u8, y in it:
                yield self.transform(u8.to(self.device)), y.to(self.device)
            return
        nxt = self._stage(it)
        while nxt is not None:
            u8, y, ev = nxt
            nxt = self._stage(it)                      # next H2D overlaps this step
            torch.cuda.current_stream(self.device).wait_event(ev)
            u8.record_stream(torch.cuda.current_stream(self.device))
            y.record_stream(torch.cuda.current_stream(self.device))
            yield self.transform(u8), y

    def _stage(self, it):
        try:
            u8, y = next(it)
        except StopIteration:
            return None
        with torch.cuda.stream(self.copy_stream):
            u8d = u8.to(self.device, non_blocking=True)
            yd = y.to(self.device, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.copy_stream)
        return u8d, yd, ev


class SyntheticLoader:
    """Synthetic batches through the same GPU transform."""

    def __init__(self, source, steps: int, transform: InputTransform):
        self.source, self.steps, self.transform = source, steps, transform

    def __len__(self):
        return self.steps

    def __iter__(self):
        for u8, y in self.source.batches(self.steps):
            yield self.transform(u8), y
