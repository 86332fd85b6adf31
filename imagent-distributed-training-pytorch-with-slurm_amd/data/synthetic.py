"""Synthetic ImageNet-shaped data (BASELINE.json: synthetic 3x224x224).

The images are uint8 HWC - exactly what the real pipeline hands to the GPU -
generated once ON the device from a seeded generator, so every training step
still runs the full GPU input path (normalise kernel -> NHWC bf16) but no host
decode or H2D copy. Labels are uniform over the classes. A pool of a few
distinct batches is cycled so consecutive steps do not see identical data.

``task='colour'`` makes the data LEARNABLE (convergence checks without
ImageNet): every class owns a mean RGB colour and a stripe orientation drawn
from a generator that depends only on the class count, so train and val sets
(different seeds) share the class -> appearance map, and images are that
colour plus stripes plus per-pixel noise.
"""

from __future__ import annotations

from typing import Iterator, Optional, Tuple

import torch


class SyntheticImageNet:
    def __init__(self, num_items: int, image_size: int = 224, num_classes: int = 1000,
                 batch_size: int = 256, device="cpu", seed: int = 0, pool_batches: int = 4,
                 rank: int = 0, task: str = "random"):
        self.n = int(num_items)
        self.size = image_size
        self.num_classes = num_classes
        self.batch = batch_size
        self.device = torch.device(device)
        g = torch.Generator(device="cpu")
        g.manual_seed(seed * 1000003 + rank)
        pb = max(1, pool_batches)
        # generate on CPU with a fixed generator (device-independent content), move once
        if task == "random":
            self.images = torch.randint(0, 256, (pb, batch_size, image_size, image_size, 3), generator=g,
                                        dtype=torch.uint8).to(self.device)
            self.labels = torch.randint(0, num_classes, (pb, batch_size), generator=g).to(self.device)
        elif task == "colour":
            self.labels = torch.randint(0, num_classes, (pb, batch_size), generator=g)
            gc = torch.Generator(device="cpu")
            gc.manual_seed(7919 * num_classes + 17)  # class appearance: independent of seed / rank
            colour = 48.0 + 160.0 * torch.rand(num_classes, 3, generator=gc)
            horiz = torch.rand(num_classes, generator=gc) < 0.5
            ramp = (torch.arange(image_size) // 4 % 2).float() * 40.0 - 20.0
            stripes_h = ramp.view(image_size, 1).expand(image_size, image_size)
            stripes_v = ramp.view(1, image_size).expand(image_size, image_size)
            lab = self.labels
            img = colour[lab].view(pb, batch_size, 1, 1, 3) + torch.where(
                horiz[lab].view(pb, batch_size, 1, 1), stripes_h, stripes_v).unsqueeze(-1)
            img = img + 24.0 * torch.randn(pb, batch_size, image_size, image_size, 3, generator=g)
            self.images = img.round().clamp(0, 255).to(torch.uint8).to(self.device)
            self.labels = self.labels.to(self.device)
        else:
            raise ValueError(f"unknown synthetic task {task!r}")
        self.classes = [str(i) for i in range(num_classes)]

    def __len__(self):
        return self.n

    def num_batches(self) -> int:
        return (self.n + self.batch - 1) // self.batch

    def batches(self, n: Optional[int] = None) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        n = self.num_batches() if n is None else n
        pb = self.images.shape[0]
        for i in range(n):
            yield self.images[i % pb], self.labels[i % pb]
