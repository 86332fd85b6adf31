"""ILSVRC2012 devkit + archives -> torchvision's ImageNet layout (imagenet.py:293-296).

A synthetic devkit (meta.mat with leaf and non-leaf synsets, validation ground
truth) and synthetic train / val archives of tiny images; the real files are
not available here (parity with torchvision's parser: same fields, same
leaf-only class list, same sorted-file -> ground-truth-line mapping)."""

import io
import os
import tarfile

import numpy as np
import pytest


def _tar_add(t, name, data):
    ti = tarfile.TarInfo(name)
    ti.size = len(data)
    t.addfile(ti, io.BytesIO(data))


def _png(seed):
    from PIL import Image
    b = io.BytesIO()
    Image.fromarray(np.full((6, 6, 3), seed * 20 % 256, dtype=np.uint8)).save(b, format="PNG")
    return b.getvalue()


def _make(root):
    import scipy.io
    wnids = ["n01440764", "n01443537", "n01484850"]
    dt = [("ILSVRC2012_ID", "O"), ("WNID", "O"), ("words", "O"), ("num_children", "O")]
    syn = np.array([(1, wnids[0], "tench, Tinca tinca", 0), (2, wnids[1], "goldfish, Carassius auratus", 0),
                    (3, wnids[2], "great white shark", 0), (1001, "n00000001", "fish", 3)], dtype=dt)
    mat = io.BytesIO()
    scipy.io.savemat(mat, {"synsets": syn})
    gt = [2, 1, 3, 2, 1]  # ILSVRC ids of val images 1..5
    with tarfile.open(os.path.join(root, "ILSVRC2012_devkit_t12.tar.gz"), "w:gz") as t:
        _tar_add(t, "ILSVRC2012_devkit_t12/data/meta.mat", mat.getvalue())
        _tar_add(t, "ILSVRC2012_devkit_t12/data/ILSVRC2012_validation_ground_truth.txt",
                 "\n".join(map(str, gt)).encode())
    with tarfile.open(os.path.join(root, "ILSVRC2012_img_val.tar"), "w") as t:
        for i in range(5):
            _tar_add(t, f"ILSVRC2012_val_{i + 1:08d}.JPEG", _png(i))
    with tarfile.open(os.path.join(root, "ILSVRC2012_img_train.tar"), "w") as t:
        for c, w in enumerate(wnids):
            inner = io.BytesIO()
            with tarfile.open(fileobj=inner, mode="w") as it:
                for j in range(2):
                    _tar_add(it, f"{w}_{j}.JPEG", _png(c * 2 + j))
            _tar_add(t, f"{w}.tar", inner.getvalue())
    return wnids, gt


def test_devkit_and_archives_give_the_torchvision_layout(tmp_path):
    pytest.importorskip("scipy")
    from imagent_amd.data.imagenet import ImageNetU8
    wnids, gt = _make(str(tmp_path))
    val = ImageNetU8(str(tmp_path), "val", (6, 6))
    assert val.wnids == wnids  # 3 leaf classes, the non-leaf synset dropped
    assert val.classes[0] == ("tench", "Tinca tinca")
    # image k (sorted file order) carries the class of ground-truth line k
    got = {os.path.basename(p): y for p, y in val.samples}
    for k, g in enumerate(gt):
        assert got[f"ILSVRC2012_val_{k + 1:08d}.JPEG"] == g - 1
    train = ImageNetU8(str(tmp_path), "train", (6, 6))
    assert len(train) == 6 and train.targets == [0, 0, 1, 1, 2, 2]
    x, y = train[3]
    assert tuple(x.shape) == (6, 6, 3) and y == 1
    # second construction: layout already in place, nothing re-extracted
    assert len(ImageNetU8(str(tmp_path), "val", (6, 6))) == 5


def _prep_worker(rank, root, outdir):
    from imagent_amd.data.devkit import prepare
    for split in ("train", "val"):
        prepare(root, split)
    open(os.path.join(outdir, f"ok{rank}"), "w").close()


def test_concurrent_ranks_prepare_once(tmp_path):
    """every rank calls prepare() at once (no rank gating in the engine); the file
    lock lets one do the work and the others find the finished layout."""
    pytest.importorskip("scipy")
    import torch.multiprocessing as mp
    from imagent_amd.data.imagenet import ImageNetU8
    root = tmp_path / "in"
    root.mkdir()
    wnids, gt = _make(str(root))
    mp.start_processes(_prep_worker, args=(str(root), str(tmp_path)), nprocs=3, start_method="spawn", join=True)
    assert all(os.path.exists(tmp_path / f"ok{r}") for r in range(3))
    val = ImageNetU8(str(root), "val", (6, 6))
    assert len(val) == 5 and sorted(os.listdir(root / "val")) == sorted(set(wnids))
    assert len(ImageNetU8(str(root), "train", (6, 6))) == 6
    assert not any(n.endswith(".partial") for n in os.listdir(root))


def test_interrupted_val_sort_resumes_from_its_plan(tmp_path):
    """A sort interrupted after some moves resumes from the written plan: the remaining flat
    files keep the class that their position in the ORIGINAL sorted listing gives them."""
    pytest.importorskip("scipy")
    import json
    import tarfile as tf
    from imagent_amd.data.devkit import prepare
    from imagent_amd.data.imagenet import ImageNetU8
    wnids, gt = _make(str(tmp_path))
    prepare(str(tmp_path), "train")  # writes meta.bin
    d = tmp_path / "val"
    d.mkdir()
    with tf.open(tmp_path / "ILSVRC2012_img_val.tar") as t:
        t.extractall(d)
    names = sorted(os.listdir(d))
    plan = [[n, wnids[g - 1]] for n, g in zip(names, gt)]
    (d / ".sort_plan.json").write_text(json.dumps(plan))
    for n, w in plan[:2]:  # the first two moves happened before the "crash"
        (d / w).mkdir(exist_ok=True)
        os.rename(d / n, d / w / n)
    prepare(str(tmp_path), "val")
    assert not (d / ".sort_plan.json").exists()
    got = {os.path.basename(p): y for p, y in ImageNetU8(str(tmp_path), "val", (6, 6)).samples}
    for k, g in enumerate(gt):
        assert got[f"ILSVRC2012_val_{k + 1:08d}.JPEG"] == g - 1


def test_prepared_tree_on_read_only_root(tmp_path):
    """a tree already in class-folder layout on a read-only mount (shared SLURM storage)
    needs no lock file: prepare() returns before opening one, and the dataset constructs."""
    pytest.importorskip("scipy")
    from imagent_amd.data.devkit import prepare
    from imagent_amd.data.imagenet import ImageNetU8
    root = tmp_path / "ro"
    root.mkdir()
    _make(str(root))
    for split in ("train", "val"):
        prepare(str(root), split)
    os.remove(root / ".imagent_prepare.lock")
    os.chmod(root, 0o555)
    try:
        if os.access(root, os.W_OK):  # running as root: permissions do not bind, check the no-lock path directly
            prepare(str(root), "val")
            assert not os.path.exists(root / ".imagent_prepare.lock")
        assert len(ImageNetU8(str(root), "val", (6, 6))) == 5
        assert len(ImageNetU8(str(root), "train", (6, 6))) == 6
        assert not os.path.exists(root / ".imagent_prepare.lock")
    finally:
        os.chmod(root, 0o755)
