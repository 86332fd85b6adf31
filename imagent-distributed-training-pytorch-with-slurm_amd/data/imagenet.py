"""ImageNet / ImageFolder sources.

Reference: ``datasets.ImageNet(root=<cwd>/../data/imagenet, split, transform)``
(``imagenet.py:287-298``) with ``Resize((448,448)) -> ToTensor ->
Normalize((.5,.5,.5),(.5,.5,.5))`` for both splits (``imagenet.py:280-283``).

MI355X split of that work: the host only decodes the JPEG and resizes it to
a uint8 HWC array (PIL, in DataLoader worker processes); the float
conversion + normalisation (+ optional crop / flip) runs on the GPU in one
HIP kernel after a 4x smaller uint8 H2D copy (:mod:`.loader`).

Index semantics follow torchvision's ImageFolder: classes = sorted wnid
sub-directories, samples = files of each class in ``sorted(os.walk)`` order
with the usual image extensions. Human-readable class names come from
``meta.bin`` (loaded with ``weights_only=True``), which :mod:`.devkit` writes
from ``ILSVRC2012_devkit_t12.tar.gz`` while it extracts the archives and
sorts the flat validation set into class folders, as torchvision does.
"""

from __future__ import annotations

import os
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

IMG_EXTENSIONS = (".jpg", ".jpeg", ".png", ".ppm", ".bmp", ".pgm", ".tif", ".tiff", ".webp")


def find_classes(directory: str) -> Tuple[List[str], dict]:
    classes = sorted(e.name for e in os.scandir(directory) if e.is_dir())
    if not classes:
        raise FileNotFoundError(f"no class folders in {directory}")
    return classes, {c: i for i, c in enumerate(classes)}


def make_index(directory: str, class_to_idx: dict) -> List[Tuple[str, int]]:
    out = []
    for cls in sorted(class_to_idx):
        d = os.path.join(directory, cls)
        for root, _, fnames in sorted(os.walk(d, followlinks=True)):
            for f in sorted(fnames):
                if f.lower().endswith(IMG_EXTENSIONS):
                    out.append((os.path.join(root, f), class_to_idx[cls]))
    return out


def load_meta(root: str) -> Optional[dict]:
    p = os.path.join(root, "meta.bin")
    if not os.path.exists(p):
        return None
    try:
        wnid_to_classes, _ = torch.load(p, weights_only=True)
        return wnid_to_classes
    except Exception:
        return None


def decode_resize(path: str, size: Tuple[int, int]) -> np.ndarray:
    """PIL decode -> RGB -> bilinear resize (antialiased, as torchvision's
    Resize on PIL images) -> uint8 HWC."""
    from PIL import Image
    with open(path, "rb") as f:
        img = Image.open(f)
        img = img.convert("RGB")
        if img.size != (size[1], size[0]):
            img = img.resize((size[1], size[0]), Image.BILINEAR)
        return np.array(img, dtype=np.uint8)  # writable copy


class ImageFolderU8(torch.utils.data.Dataset):
    """Yields (uint8 [H, W, 3] tensor, label)."""

    def __init__(self, root: str, size: Tuple[int, int] = (448, 448)):
        self.root = root
        self.size = tuple(size)
        self.classes, self.class_to_idx = find_classes(root)
        self.samples = make_index(root, self.class_to_idx)
        if not self.samples:
            raise FileNotFoundError(f"no images under {root}")
        self.targets = [s[1] for s in self.samples]

    def __len__(self):
        return len(self.samples)

    def __getitem__(self, i):
        path, y = self.samples[i]
        return torch.from_numpy(decode_resize(path, self.size)), y


class ImageNetU8(ImageFolderU8):
    """``datasets.ImageNet(root, split)`` layout: ``root/{train,val}/<wnid>/``."""

    def __init__(self, root: str, split: str = "train", size: Tuple[int, int] = (448, 448)):
        if split not in ("train", "val"):
            raise ValueError(split)
        from .devkit import prepare
        prepare(root, split)  # archives / devkit -> <split>/<wnid>/ (torchvision's first-use work)
        super().__init__(os.path.join(root, split), size)
        self.split = split
        self.wnids = list(self.classes)
        meta = load_meta(root)
        if meta:
            self.classes = [meta.get(w, (w,)) for w in self.wnids]


def collate_u8(batch: Sequence[Tuple[torch.Tensor, int]]):
    imgs = torch.stack([b[0] for b in batch])
    labels = torch.tensor([b[1] for b in batch], dtype=torch.int64)
    return imgs, labels
