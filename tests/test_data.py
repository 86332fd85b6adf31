"""ImageFolder index, decode/resize and the CPU input transform."""

import os

import numpy as np
import pytest
import torch

from imagent_amd.data.imagenet import ImageNetU8, collate_u8, decode_resize
from imagent_amd.data.loader import DeviceLoader, InputTransform
from imagent_amd.data.synthetic import SyntheticImageNet
from imagent_amd.parallel.sampler import ShardSampler


@pytest.fixture()
def tiny_imagenet(tmp_path):
    from PIL import Image
    rng = np.random.default_rng(0)
    for split, n in (("train", 3), ("val", 2)):
        for wnid in ("n02", "n01", "n03"):
            d = tmp_path / split / wnid
            d.mkdir(parents=True)
            for i in range(n):
                a = rng.integers(0, 256, (20 + i, 30, 3), dtype=np.uint8)
                Image.fromarray(a).save(d / f"img_{i}.JPEG", quality=95)
    (tmp_path / "train" / "n01" / "notes.txt").write_text("ignored")
    return tmp_path


def test_index_order_and_classes(tiny_imagenet):
    ds = ImageNetU8(str(tiny_imagenet), "train", (16, 16))
    assert ds.wnids == ["n01", "n02", "n03"]            # sorted wnids (ImageFolder)
    assert len(ds) == 9
    assert [os.path.basename(p) for p, _ in ds.samples[:3]] == ["img_0.JPEG", "img_1.JPEG", "img_2.JPEG"]
    assert ds.targets == [0, 0, 0, 1, 1, 1, 2, 2, 2]
    x, y = ds[4]
    assert x.shape == (16, 16, 3) and x.dtype == torch.uint8 and y == 1


def test_decode_resize_matches_pil_bilinear(tiny_imagenet):
    from PIL import Image
    p = str(tiny_imagenet / "val" / "n01" / "img_0.JPEG")
    a = decode_resize(p, (12, 8))
    ref = np.asarray(Image.open(p).convert("RGB").resize((8, 12), Image.BILINEAR))
    assert a.shape == (12, 8, 3) and np.array_equal(a, ref)


def test_cpu_transform_is_totensor_normalize():
    u8 = torch.randint(0, 256, (2, 4, 5, 3), dtype=torch.uint8)
    x = InputTransform("torch", (4, 5))(u8)
    ref = (u8.permute(0, 3, 1, 2).float() / 255 - 0.5) / 0.5
    torch.testing.assert_close(x, ref)


def test_loader_iterates_shard(tiny_imagenet):
    ds = ImageNetU8(str(tiny_imagenet), "val", (8, 8))
    s = ShardSampler(len(ds), 2, 1, shuffle=False)
    dl = DeviceLoader(ds, s, 2, InputTransform("torch", (8, 8)), "cpu", workers=0)
    batches = list(dl)
    assert len(batches) == len(dl) == 2
    assert batches[0][0].shape == (2, 3, 8, 8)
    ys = torch.cat([b[1] for b in batches]).tolist()
    assert ys == [ds.targets[i] for i in list(s)]


def test_synthetic_is_deterministic_per_rank():
    a = SyntheticImageNet(100, 16, 10, 4, "cpu", seed=1, rank=0)
    b = SyntheticImageNet(100, 16, 10, 4, "cpu", seed=1, rank=0)
    c = SyntheticImageNet(100, 16, 10, 4, "cpu", seed=1, rank=1)
    assert torch.equal(a.images, b.images) and not torch.equal(a.images, c.images)
    assert a.num_batches() == 25
    x, y = next(a.batches(1))
    assert x.shape == (4, 16, 16, 3) and y.max() < 10


def test_collate():
    imgs, labels = collate_u8([(torch.zeros(2, 2, 3, dtype=torch.uint8), 1),
                               (torch.ones(2, 2, 3, dtype=torch.uint8), 4)])
    assert imgs.shape == (2, 2, 2, 3) and labels.tolist() == [1, 4]


def test_mix_pool_is_byte_capped_and_chunked(monkeypatch):
    """task='mix' renders its resident pool in chunks of whole batches, and the trainer caps the pool by bytes
    (the CLI defaults asked for ~316 GB of images)."""
    from imagent_amd.data import synthetic as S
    assert S.mix_pool_cap(128, 448, budget_gb=16) == (16 << 30) // (128 * 448 * 448 * 3)
    assert S.mix_pool_cap(128, 448, budget_gb=1e-9) == 1
    whole = SyntheticImageNet(5 * 8, 16, 10, 8, "cpu", seed=3, pool_batches=5, task="mix")
    monkeypatch.setattr(S, "MIX_CHUNK_BYTES", 4 * 8 * 16 * 16 * 3 * 2)  # 2 batches per chunk
    chunked = SyntheticImageNet(5 * 8, 16, 10, 8, "cpu", seed=3, pool_batches=5, task="mix")
    assert chunked.images.shape == (5, 8, 16, 16, 3) and chunked.images.dtype == torch.uint8
    assert torch.equal(whole.labels, chunked.labels)
    # same class -> appearance map and value range, a different per-chunk noise draw
    assert abs(whole.images.float().mean().item() - chunked.images.float().mean().item()) < 4.0


def test_cpu_transform_resize_is_interpolate():
    """--record-resize on the torch path: bilinear (align_corners=False) then ToTensor/Normalize."""
    import torch.nn.functional as F
    u8 = torch.randint(0, 256, (2, 20, 30, 3), dtype=torch.uint8)
    x = InputTransform("torch", (40, 24), resize=True)(u8)
    ref = F.interpolate(u8.permute(0, 3, 1, 2).float(), size=(40, 24), mode="bilinear", align_corners=False)
    assert x.shape == (2, 3, 40, 24)
    assert torch.allclose(x, (ref / 255.0 - 0.5) / 0.5, atol=1e-5)
