"""ILSVRC2012 archives and devkit, as ``torchvision.datasets.ImageNet`` handles them.

The reference builds its datasets with ``datasets.ImageNet(root, split=...)``
(``imagenet.py:293-296``), which on first use

* parses ``ILSVRC2012_devkit_t12.tar.gz`` (``data/meta.mat`` -> ILSVRC2012 id
  -> wnid -> human-readable class names; ``data/ILSVRC2012_validation_ground
  _truth.txt`` -> the wnid of every validation image),
* extracts ``ILSVRC2012_img_train.tar`` (a tar of per-class tars) into
  ``train/<wnid>/`` and ``ILSVRC2012_img_val.tar`` into ``val/``, then moves the
  flat validation images into ``val/<wnid>/`` folders,
* caches ``(wnid_to_classes, val_wnids)`` in ``meta.bin``.

Same here, with safe readers only: ``scipy.io.loadmat`` for the MATLAB file,
``tarfile`` with the ``data`` extraction filter (no absolute paths, no links
out of the tree), and ``meta.bin`` written with ``torch.save`` of plain
containers so :func:`imagenet.load_meta` reads it with ``weights_only=True``.
"""

from __future__ import annotations

import contextlib
import io
import json
import os
import shutil
import tarfile
from typing import Dict, List, Tuple

DEVKIT = "ILSVRC2012_devkit_t12.tar.gz"
TRAIN_TAR = "ILSVRC2012_img_train.tar"
VAL_TAR = "ILSVRC2012_img_val.tar"
META_FILE = "meta.bin"


def _extract(tar: tarfile.TarFile, dest: str) -> None:
    try:
        tar.extractall(dest, filter="data")  # refuses absolute paths / escaping links
    except TypeError:  # an interpreter without extraction filters: check the members ourselves
        root = os.path.realpath(dest)
        for m in tar.getmembers():
            p = os.path.realpath(os.path.join(dest, m.name))
            if not p.startswith(root + os.sep) or m.issym() or m.islnk() or m.isdev():
                raise RuntimeError(f"unsafe archive member {m.name!r}")
        tar.extractall(dest)


def parse_devkit(path: str) -> Tuple[Dict[str, Tuple[str, ...]], List[str]]:
    """(wnid -> class names, wnid of every validation image in file order)."""
    import scipy.io
    with tarfile.open(path, "r:*") as t:
        def member(suffix):
            for m in t.getmembers():
                if m.name.endswith(suffix):
                    return t.extractfile(m).read()
            raise FileNotFoundError(f"{suffix} not in {path}")
        meta = scipy.io.loadmat(io.BytesIO(member("data/meta.mat")), squeeze_me=True)["synsets"]
        gt = member("data/ILSVRC2012_validation_ground_truth.txt").decode().split()
    idx_to_wnid, wnid_to_classes = {}, {}
    for s in meta:
        if int(s["num_children"]) != 0:  # only the 1000 leaf synsets are classes
            continue
        wnid = str(s["WNID"])
        idx_to_wnid[int(s["ILSVRC2012_ID"])] = wnid
        wnid_to_classes[wnid] = tuple(c.strip() for c in str(s["words"]).split(","))
    return wnid_to_classes, [idx_to_wnid[int(i)] for i in gt]


def _has_class_dirs(d: str) -> bool:
    return os.path.isdir(d) and any(e.is_dir() for e in os.scandir(d))


@contextlib.contextmanager
def _lock(root: str):
    """Exclusive POSIX record lock on ``root/.imagent_prepare.lock``: every rank of a job (also on
    other nodes sharing the file system) calls :func:`prepare`; the first does the work, the others
    wait here and then find the split ready."""
    import fcntl
    fd = os.open(os.path.join(root, ".imagent_prepare.lock"), os.O_RDWR | os.O_CREAT, 0o644)
    try:
        fcntl.lockf(fd, fcntl.LOCK_EX)
        yield
    finally:
        try:
            fcntl.lockf(fd, fcntl.LOCK_UN)
        finally:
            os.close(fd)


def _prepare_train(root: str, d: str) -> None:
    # extract into a scratch dir and rename it into place when complete: an interrupted
    # extraction never leaves a partial train/ that a later run would take as complete
    tmp = os.path.join(root, ".train.partial")
    shutil.rmtree(tmp, ignore_errors=True)
    os.makedirs(tmp)
    with tarfile.open(os.path.join(root, TRAIN_TAR)) as t:
        _extract(t, tmp)
    for f in sorted(os.listdir(tmp)):  # one tar per class
        if f.endswith(".tar"):
            cdir = os.path.join(tmp, f[:-4])
            os.makedirs(cdir, exist_ok=True)
            with tarfile.open(os.path.join(tmp, f)) as t:
                _extract(t, cdir)
            os.remove(os.path.join(tmp, f))
    if os.path.isdir(d):
        os.rmdir(d)  # an empty leftover only (_has_class_dirs was false); refuses to drop files
    os.rename(tmp, d)


def _sort_val(d: str, meta_path: str) -> None:
    """Move the flat validation images into ``<wnid>/`` folders. The move plan is written first
    (``.sort_plan.json``, sorted file order -> ground-truth wnid) and removed last, so an
    interrupted sort resumes from the plan instead of re-deriving the order from a half-moved
    directory."""
    import torch
    plan_path = os.path.join(d, ".sort_plan.json")
    if os.path.exists(plan_path):
        with open(plan_path) as f:
            plan = json.load(f)
    else:
        _, val_wnids = torch.load(meta_path, weights_only=True)
        images = sorted(f for f in os.listdir(d) if os.path.isfile(os.path.join(d, f)) and not f.startswith("."))
        if len(images) != len(val_wnids):
            raise RuntimeError(f"{len(images)} validation images but {len(val_wnids)} ground-truth labels")
        plan = list(zip(images, val_wnids))
        with open(plan_path + ".tmp", "w") as f:
            json.dump(plan, f)
        os.replace(plan_path + ".tmp", plan_path)
    for w in {w for _, w in plan}:
        os.makedirs(os.path.join(d, w), exist_ok=True)
    for img, w in plan:
        src = os.path.join(d, img)
        if os.path.exists(src):
            shutil.move(src, os.path.join(d, w, img))
    os.remove(plan_path)


def _ready(root: str, split: str) -> bool:
    """Is ``root/<split>`` already in class-folder layout, with nothing left to do for it?"""
    d = os.path.join(root, split)
    if not _has_class_dirs(d) or os.path.exists(os.path.join(d, ".sort_plan.json")):
        return False
    # the meta file is only produced when a devkit is there to produce it from
    return os.path.exists(os.path.join(root, META_FILE)) or not os.path.exists(os.path.join(root, DEVKIT))


def prepare(root: str, split: str) -> None:
    """Bring ``root/<split>`` into the ``<wnid>/`` folder layout from the
    archives / devkit that sit in ``root`` (no-op when it already is).

    Safe to call from every rank at once (a file lock serialises the work) and
    after an interrupted run (scratch-dir extraction, resumable val sort)."""
    if not os.path.isdir(root):
        return
    if _ready(root, split):  # nothing to do: no lock (a prepared tree on a read-only mount stays usable)
        return
    with _lock(root):
        import torch
        dk = os.path.join(root, DEVKIT)
        meta_path = os.path.join(root, META_FILE)
        if not os.path.exists(meta_path) and os.path.exists(dk):
            wnid_to_classes, val_wnids = parse_devkit(dk)
            torch.save((wnid_to_classes, val_wnids), meta_path + ".tmp")
            os.replace(meta_path + ".tmp", meta_path)
        d = os.path.join(root, split)
        if split == "train" and not _has_class_dirs(d) and os.path.exists(os.path.join(root, TRAIN_TAR)):
            _prepare_train(root, d)
        if split == "val":
            pending = os.path.exists(os.path.join(d, ".sort_plan.json"))
            if not _has_class_dirs(d) or pending:
                if not os.path.isdir(d) and os.path.exists(os.path.join(root, VAL_TAR)):
                    tmp = os.path.join(root, ".val.partial")
                    shutil.rmtree(tmp, ignore_errors=True)
                    os.makedirs(tmp)
                    with tarfile.open(os.path.join(root, VAL_TAR)) as t:
                        _extract(t, tmp)
                    os.rename(tmp, d)
                if os.path.isdir(d):
                    if not os.path.exists(meta_path):
                        raise FileNotFoundError(f"{d} holds flat images: the devkit {DEVKIT} (or {META_FILE}) is "
                                                "needed to sort them into class folders")
                    _sort_val(d, meta_path)
