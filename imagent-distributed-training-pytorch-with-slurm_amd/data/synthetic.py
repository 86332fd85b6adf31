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
colour plus stripes plus per-pixel noise. Every path reaches 100 % on it.

``task='mix'`` is the one that can tell numerics apart: classes are overlapping Gaussians in the coefficient
space of 32 smooth random bases (:func:`mix_render`), so the Bayes-optimal top-1 is ~85 % (100 classes) and a
short run of the fp32 oracle ends well below it; the pool holds every distinct training batch.
"""

from __future__ import annotations

import math
from typing import Iterator, Optional, Tuple

import torch
import torch.nn.functional as F

# task='mix': class-coefficient noise (in units of the class-mean spread). With 100 classes in 32 dimensions the
# Bayes-optimal (nearest-mean) accuracy is mix_bayes_accuracy(100) = 0.85 at 1.4 -- the fp32 oracle stays well
# below 100 % top-1 within a short run, so a numerics regression shows as a lower curve
MIX_SIGMA = 1.4
MIX_DIM = 32
MIX_CHUNK_BYTES = 1 << 30  # host fp32 working set of one render chunk


def mix_pool_cap(batch_size: int, image_size: int, budget_gb: Optional[float] = None) -> int:
    """Most batches a resident task='mix' pool may hold: IMAGENT_MIX_POOL_GB (default 16) of uint8 images."""
    import os
    gb = float(os.environ.get("IMAGENT_MIX_POOL_GB", "16")) if budget_gb is None else budget_gb
    return max(1, int(gb * (1 << 30)) // (batch_size * image_size * image_size * 3))


def _mix_model(num_classes: int, image_size: int):
    """The class -> appearance map of task='mix' (depends only on the class count and size): MIX_DIM smooth
    random RGB bases (8x8x3 Gaussian fields, bilinearly upsampled, unit RMS) and per-class mean coefficients
    ~ N(0, I)."""
    gc = torch.Generator(device="cpu")
    gc.manual_seed(104729 * num_classes + 31)
    low = torch.randn(MIX_DIM, 3, 8, 8, generator=gc)
    basis = F.interpolate(low, size=(image_size, image_size), mode="bilinear", align_corners=False)
    basis = basis / basis.pow(2).mean(dim=(1, 2, 3), keepdim=True).sqrt()
    means = torch.randn(num_classes, MIX_DIM, generator=gc)
    return basis.permute(0, 2, 3, 1).reshape(MIX_DIM, -1), means  # [J][S*S*3] (HWC), [K][J]


def mix_render(labels: torch.Tensor, image_size: int, num_classes: int, g: torch.Generator,
               sigma: float = MIX_SIGMA) -> torch.Tensor:
    """uint8 [n, S, S, 3] images of task='mix': coefficients a = mean[label] + sigma z (z ~ N(0, I), a fresh draw
    per image), image = 128 + 40 a . basis / sqrt(J (1 + sigma^2)) + 10 N(0, 1) per pixel. Classes are Gaussians
    with a shared covariance in coefficient space: learnable by a linear read-out of the bases, with a Bayes error
    set by sigma (classes overlap), so accuracy measures how well training went rather than saturating."""
    basis, means = _mix_model(num_classes, image_size)
    n = labels.numel()
    a = means[labels] + sigma * torch.randn(n, MIX_DIM, generator=g)
    img = 128.0 + (40.0 / math.sqrt(MIX_DIM * (1.0 + sigma * sigma))) * (a @ basis)
    img = img + 10.0 * torch.randn(img.shape, generator=g)
    return img.round().clamp(0, 255).to(torch.uint8).view(n, image_size, image_size, 3)


def mix_bayes_accuracy(num_classes: int, sigma: float = MIX_SIGMA, n: int = 20000, seed: int = 0) -> float:
    """Monte-Carlo accuracy of the Bayes-optimal classifier of task='mix' in coefficient space (nearest class
    mean; shared isotropic covariance, uniform labels): an upper bound for any network on these images (pixel
    noise and clamping only lose information)."""
    _, means = _mix_model(num_classes, 8)
    g = torch.Generator(device="cpu")
    g.manual_seed(seed)
    y = torch.randint(0, num_classes, (n,), generator=g)
    a = means[y] + sigma * torch.randn(n, MIX_DIM, generator=g)
    pred = torch.cdist(a, means).argmin(dim=1)
    return float((pred == y).float().mean())


class SyntheticImageNet:
    def __init__(self, num_items: int, image_size: int = 224, num_classes: int = 1000,
                 batch_size: int = 256, device="cpu", seed: int = 0, pool_batches: int = 4,
                 rank: int = 0, task: str = "random", mix_sigma: float = MIX_SIGMA):
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
        elif task == "mix":
            self.labels = torch.randint(0, num_classes, (pb, batch_size), generator=g)
            # rendered in chunks of whole batches (mix_render's fp32 intermediate is 4x the uint8 images) straight
            # into the resident device pool
            self.images = torch.empty((pb, batch_size, image_size, image_size, 3), dtype=torch.uint8,
                                      device=self.device)
            per = max(1, MIX_CHUNK_BYTES // (4 * batch_size * image_size * image_size * 3))
            for b0 in range(0, pb, per):
                b1 = min(pb, b0 + per)
                img = mix_render(self.labels[b0:b1].reshape(-1), image_size, num_classes, g, sigma=mix_sigma)
                self.images[b0:b1].copy_(img.view(b1 - b0, batch_size, image_size, image_size, 3))
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
