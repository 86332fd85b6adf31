"""Packed uint8 image records and the native gather loader.

The reference decodes, resizes (448x448), converts and normalises every image
on every epoch in 10 DataLoader worker processes per rank
(``imagenet.py:280-283, 350-359``; 1 CPU per task, ``imagenet.sh:10``) --
SURVEY §6 reads its throughput as input-bound. Here decode + resize run ONCE
(:func:`write_records`, :func:`convert_imagefolder`,
``python -m imagent_amd.data.records``) into a file of fixed-size uint8 rows;
per step the C++ runtime (``csrc/runtime/records.cpp``) gathers the sampler's
rows from the memory-mapped file into pinned host memory on a thread pool,
the H2D copy runs on a HIP copy stream and one GPU kernel normalises
(:class:`~.loader.InputTransform`). Nothing per-sample runs in Python.

File layout (little endian): 64-B header ``IMREC001 | n | H | W | C | classes |
images_off | 3 x reserved``, int32 labels[n], zero pad to 4 KiB, uint8
images[n][H][W][C].
"""

from __future__ import annotations

import argparse
import ctypes as C
import os
import struct
from typing import Iterable, Iterator, Optional, Sequence, Tuple

import numpy as np
import torch

MAGIC = b"IMREC001"
HEADER = struct.Struct("<8sqiiiiq3q")
ALIGN = 4096
assert HEADER.size == 64


def _images_off(n: int) -> int:
    return (HEADER.size + 4 * n + ALIGN - 1) // ALIGN * ALIGN


def write_records(path: str, items: Iterable[Tuple[np.ndarray, int]], n: int, size: Tuple[int, int],
                  classes: int, channels: int = 3) -> None:
    """Write ``n`` (uint8 [H, W, C] image, label) pairs to ``path`` (atomic rename)."""
    h, w = size
    rec = h * w * channels
    off = _images_off(n)
    labels = np.zeros(n, dtype=np.int32)
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        f.write(HEADER.pack(MAGIC, n, h, w, channels, classes, off, 0, 0, 0))
        f.seek(off)
        i = 0
        for img, y in items:
            if i >= n:
                raise ValueError(f"more than {n} records")
            a = np.ascontiguousarray(img, dtype=np.uint8)
            if a.shape != (h, w, channels):
                raise ValueError(f"record {i}: shape {a.shape} != {(h, w, channels)}")
            f.write(memoryview(a).cast("B"))
            labels[i] = int(y)
            i += 1
        if i != n:
            raise ValueError(f"expected {n} records, got {i}")
        f.seek(HEADER.size)
        f.write(labels.tobytes())
        f.truncate(off + n * rec)
    os.replace(tmp, path)


def _decode(job):
    from .imagenet import decode_resize
    path, size = job
    return decode_resize(path, size)


def convert_imagefolder(ds, path: str, workers: int = 8) -> None:
    """An :class:`~.imagenet.ImageFolderU8` / ``ImageNetU8`` -> record file, in
    index order: PIL decode + bilinear resize once, in ``workers`` processes."""
    jobs = [(p, ds.size) for p, _ in ds.samples]
    labels = [y for _, y in ds.samples]

    def items(images):
        return zip(images, labels)

    if workers > 0:
        import multiprocessing as mp
        with mp.get_context("fork").Pool(workers) as pool:
            write_records(path, items(pool.imap(_decode, jobs, chunksize=16)), len(jobs), ds.size,
                          len(ds.classes))
    else:
        write_records(path, items(map(_decode, jobs)), len(jobs), ds.size, len(ds.classes))


class RecordFile:
    """A memory-mapped record file with a native gather thread pool."""

    def __init__(self, path: str, threads: int = 8, slots: int = 3):
        from ..ops import _lib
        self.L = _lib.runtime()
        self.path = path
        self.slots = max(2, int(slots))
        self.h = self.L.imr_records_open(path.encode(), int(threads), self.slots)
        if not self.h:
            raise ValueError(f"{path}: missing, truncated or not an {MAGIC.decode()} record file")
        info = (C.c_int64 * 5)()
        self.L.imr_records_info(self.h, info)
        self.n = int(info[0])
        self.shape = (int(info[1]), int(info[2]), int(info[3]))
        self.num_classes = int(info[4])
        lab = np.empty(self.n, dtype=np.int32)
        self.L.imr_records_labels(self.h, lab.ctypes.data)
        self.targets = lab

    def __len__(self) -> int:
        return self.n

    def submit(self, slot: int, idx: torch.Tensor, images: torch.Tensor, labels: Optional[torch.Tensor]) -> None:
        idx = idx.to(torch.int64).contiguous()
        cnt = idx.numel()
        assert images.is_contiguous() and images.dtype == torch.uint8 and images.numel() >= cnt * int(
            np.prod(self.shape))
        assert labels is None or (labels.dtype == torch.int64 and labels.numel() >= cnt)
        rc = self.L.imr_records_submit(self.h, slot, idx.data_ptr(), cnt, images.data_ptr(),
                                       labels.data_ptr() if labels is not None else None)
        if rc != 0:
            raise RuntimeError(f"records submit: slot {slot} rc={rc}")

    def wait(self, slot: int) -> None:
        rc = self.L.imr_records_wait(self.h, slot)
        if rc == -3:
            raise IndexError(f"{self.path}: record index out of range (0..{self.n - 1})")
        if rc != 0:
            raise RuntimeError(f"records wait: slot {slot} rc={rc}")

    def gather(self, idx: Sequence[int]) -> Tuple[torch.Tensor, torch.Tensor]:
        """Synchronous gather (tests, tools): uint8 [B, H, W, C], int64 [B]."""
        idx = torch.as_tensor(idx, dtype=torch.int64)
        imgs = torch.empty((idx.numel(),) + self.shape, dtype=torch.uint8)
        labs = torch.empty(idx.numel(), dtype=torch.int64)
        self.submit(0, idx, imgs, labs)
        self.wait(0)
        return imgs, labs

    def close(self) -> None:
        if getattr(self, "h", None):
            self.L.imr_records_close(self.h)
            self.h = None

    def __del__(self):
        self.close()


class RecordLoader:
    """(model_input, labels) batches of one rank's shard of a :class:`RecordFile`.

    Slot ring: while batch k is being normalised and trained on, batch k+1
    (and up to ``slots - 2`` more) is already being gathered by the native
    pool into its own pinned buffer; a slot is refilled only after the H2D
    copy out of it (on the copy stream) has completed."""

    def __init__(self, rf: RecordFile, sampler, batch_size: int, transform, device, drop_last: bool = False):
        self.rf, self.sampler, self.batch = rf, sampler, batch_size
        self.transform, self.device = transform, torch.device(device)
        self.drop_last = drop_last
        pin = self.device.type == "cuda"
        S = rf.slots
        self.bufs = [torch.empty((batch_size,) + rf.shape, dtype=torch.uint8, pin_memory=pin) for _ in range(S)]
        self.labs = [torch.empty(batch_size, dtype=torch.int64, pin_memory=pin) for _ in range(S)]
        self.copy_stream = torch.cuda.Stream(self.device) if pin else None
        self.copied = [None] * S

    def __len__(self) -> int:
        return self.sampler.num_batches(self.batch, self.drop_last)

    def _submit(self, k: int, batches) -> None:
        s = k % len(self.bufs)
        if self.copied[s] is not None:
            self.copied[s].synchronize()  # the slot's previous H2D copy has drained
            self.copied[s] = None
        self.rf.submit(s, batches[k], self.bufs[s], self.labs[s])

    def __iter__(self) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        batches = list(self.sampler.batches(self.batch, self.drop_last))
        S, nb = len(self.bufs), len(batches)
        for k in range(min(S - 1, nb)):
            self._submit(k, batches)
        for k in range(nb):
            if k + S - 1 < nb:
                self._submit(k + S - 1, batches)  # reuses batch k-1's slot
            s = k % S
            self.rf.wait(s)
            cnt = batches[k].numel()
            u8, y = self.bufs[s][:cnt], self.labs[s][:cnt]
            if self.copy_stream is None:
                yield self.transform(u8.clone()), y.clone()
                continue
            with torch.cuda.stream(self.copy_stream):
                u8d = u8.to(self.device, non_blocking=True)
                yd = y.to(self.device, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self.copy_stream)
            self.copied[s] = ev
            cur = torch.cuda.current_stream(self.device)
            cur.wait_event(ev)
            u8d.record_stream(cur)
            yd.record_stream(cur)
            yield self.transform(u8d), yd


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="ImageNet folder -> uint8 record files (train.imrec, val.imrec)")
    ap.add_argument("--root", required=True, help="ImageNet root with train/ and val/ (imagenet.py:287)")
    ap.add_argument("--out", required=True)
    ap.add_argument("--size", type=int, default=448, help="square image size (imagenet.py:281)")
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--splits", default="train,val")
    a = ap.parse_args(argv)
    from .imagenet import ImageNetU8
    os.makedirs(a.out, exist_ok=True)
    for split in a.splits.split(","):
        ds = ImageNetU8(a.root, split, (a.size, a.size))
        dst = os.path.join(a.out, f"{split}.imrec")
        convert_imagefolder(ds, dst, a.workers)
        print(f"{split}: {len(ds)} images, {len(ds.classes)} classes -> {dst}", flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
