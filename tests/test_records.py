"""Packed uint8 record files + the native gather loader (csrc/runtime/records.cpp)."""

import os

import numpy as np
import pytest
import torch

from imagent_amd.data.loader import InputTransform
from imagent_amd.data.records import (HEADER, MAGIC, RecordFile, RecordLoader, convert_imagefolder,
                                      write_records)
from imagent_amd.parallel.sampler import ShardSampler


def _random_records(path, n=37, size=(6, 5), classes=11, seed=0):
    rng = np.random.default_rng(seed)
    imgs = rng.integers(0, 256, (n, size[0], size[1], 3), dtype=np.uint8)
    labels = rng.integers(0, classes, n)
    write_records(str(path), zip(imgs, labels), n, size, classes)
    return imgs, labels


def test_header_layout(tmp_path):
    p = tmp_path / "a.imrec"
    _random_records(p, n=3)
    raw = open(p, "rb").read()
    magic, n, h, w, c, classes, off = HEADER.unpack_from(raw)[:7]
    assert (magic, n, h, w, c, classes) == (MAGIC, 3, 6, 5, 3, 11)
    assert off % 4096 == 0 and len(raw) == off + 3 * 6 * 5 * 3


@pytest.mark.parametrize("threads", [0, 3])
def test_gather_matches_source(tmp_path, threads):
    p = tmp_path / "a.imrec"
    imgs, labels = _random_records(p)
    rf = RecordFile(str(p), threads=threads, slots=2)
    assert len(rf) == 37 and rf.shape == (6, 5, 3) and rf.num_classes == 11
    assert np.array_equal(rf.targets, labels)
    idx = [5, 0, 36, 5, 17]
    x, y = rf.gather(idx)
    assert np.array_equal(x.numpy(), imgs[idx]) and y.tolist() == labels[idx].tolist()
    rf.close()


def test_out_of_range_and_bad_files(tmp_path):
    p = tmp_path / "a.imrec"
    _random_records(p)
    rf = RecordFile(str(p), threads=2)
    with pytest.raises(IndexError):
        rf.gather([1, 37])
    x, y = rf.gather([2])  # the slot is usable again after the error
    assert y.numel() == 1
    bad = tmp_path / "bad.imrec"
    bad.write_bytes(b"NOTAREC0" + bytes(100))
    with pytest.raises(ValueError):
        RecordFile(str(bad))
    trunc = tmp_path / "trunc.imrec"
    trunc.write_bytes(open(p, "rb").read()[:-10])
    with pytest.raises(ValueError):
        RecordFile(str(trunc))
    with pytest.raises(ValueError):
        RecordFile(str(tmp_path / "missing.imrec"))


def test_loader_iterates_one_ranks_shard(tmp_path):
    p = tmp_path / "a.imrec"
    imgs, labels = _random_records(p)
    rf = RecordFile(str(p), threads=2, slots=3)
    s = ShardSampler(len(rf), 2, 1, shuffle=True, seed=3)
    s.set_epoch(4)
    dl = RecordLoader(rf, s, 4, InputTransform("torch", (6, 5)), "cpu")
    batches = list(dl)
    assert len(batches) == len(dl) == 5  # 19 samples of this rank, last batch partial
    want = s.indices().tolist()
    got_y = torch.cat([b[1] for b in batches]).tolist()
    assert got_y == labels[want].tolist()
    x = torch.cat([b[0] for b in batches])
    ref = (torch.from_numpy(imgs[want]).permute(0, 3, 1, 2).float() / 255 - 0.5) / 0.5
    torch.testing.assert_close(x, ref)


def test_convert_imagefolder_matches_decode(tmp_path):
    from PIL import Image

    from imagent_amd.data.imagenet import ImageNetU8, decode_resize
    rng = np.random.default_rng(1)
    for wnid in ("n02", "n01"):
        d = tmp_path / "train" / wnid
        d.mkdir(parents=True)
        for i in range(3):
            Image.fromarray(rng.integers(0, 256, (20 + i, 30, 3), dtype=np.uint8)).save(d / f"i{i}.JPEG")
    ds = ImageNetU8(str(tmp_path), "train", (12, 16))
    for workers in (0, 2):
        out = tmp_path / f"train{workers}.imrec"
        convert_imagefolder(ds, str(out), workers=workers)
        rf = RecordFile(str(out), threads=1)
        x, y = rf.gather(list(range(len(ds))))
        assert y.tolist() == ds.targets and rf.num_classes == 2
        for i, (path, _) in enumerate(ds.samples):
            assert np.array_equal(x[i].numpy(), decode_resize(path, (12, 16)))
        rf.close()
    assert not os.path.exists(str(tmp_path / "train0.imrec.tmp"))
