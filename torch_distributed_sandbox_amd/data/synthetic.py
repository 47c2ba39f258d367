"""Synthetic MNIST-like data, upscaled on the GPU.

The reference reads torchvision MNIST (60 000 28x28 images), resizes each one
to 3000x3000 with PIL on the CPU and copies 180 MB per batch over PCIe
(mnist_onegpu.py:51-59) — ~139 ms/image on the host, i.e. input-bound.  There
is no torchvision and no network here, so:

* :class:`SyntheticMNIST` — deterministic, seeded 28x28 uint8 images + labels.
  Each class has a fixed random "digit" template (blurred strokes); samples
  are the template with a random shift and noise, so a model can actually
  learn (loss decreases) while shapes and value ranges match MNIST.
* :class:`DeviceUpsampleLoader` — batches of 28x28 uint8 go to the GPU
  (B*784 bytes instead of B*36 MB) and are bilinearly upscaled there by the
  ``upsample_bilinear_u8`` kernel (half-pixel centres + edge clamp + round to
  uint8 + /255, i.e. PIL Resize + ToTensor).  Sharding comes from a sampler
  (``parallel.sampler.DistributedSampler``) exactly like the reference's
  DataLoader(sampler=...).
"""
from __future__ import annotations

import math
from typing import Optional, Sequence

import numpy as np
import torch

from ..ops import functional as TF

MNIST_TRAIN_SIZE = 60000


def _class_templates(num_classes: int, size: int, seed: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    t = np.zeros((num_classes, size, size), np.float32)
    yy, xx = np.mgrid[0:size, 0:size].astype(np.float32)
    for c in range(num_classes):
        for _ in range(3):  # three strokes per "digit"
            x0, y0, x1, y1 = rng.uniform(6, size - 6, 4)
            n = 24
            for s in np.linspace(0, 1, n):
                cx, cy = x0 + (x1 - x0) * s, y0 + (y1 - y0) * s
                t[c] += np.exp(-((xx - cx) ** 2 + (yy - cy) ** 2) / 3.0)
        t[c] /= t[c].max()
    return t


class SyntheticMNIST:
    """Indexable dataset of (uint8[28,28], label) pairs, fully deterministic."""

    def __init__(self, size: int = MNIST_TRAIN_SIZE, num_classes: int = 10, image_size: int = 28, seed: int = 0,
                 noise: float = 0.15):
        self.size, self.num_classes, self.image_size = size, num_classes, image_size
        self.seed = seed
        rng = np.random.default_rng(seed + 1)
        self.labels = rng.integers(0, num_classes, size=size, dtype=np.int64)
        templ = _class_templates(num_classes, image_size, seed)
        # materialise all images once (60000*784 B = 47 MB)
        imgs = np.empty((size, image_size, image_size), np.uint8)
        chunk = 4096
        for s in range(0, size, chunk):
            e = min(size, s + chunk)
            n = e - s
            shifts = rng.integers(-2, 3, size=(n, 2))
            base = templ[self.labels[s:e]]
            out = np.empty_like(base)
            for i in range(n):
                out[i] = np.roll(base[i], tuple(shifts[i]), axis=(0, 1))
            out = out + noise * rng.standard_normal(out.shape).astype(np.float32)
            imgs[s:e] = np.clip(out * 255.0, 0, 255).astype(np.uint8)
        self.images = imgs

    def __len__(self) -> int:
        return self.size

    def __getitem__(self, i):
        return self.images[i], int(self.labels[i])

    def batch(self, indices: Sequence[int]):
        idx = np.asarray(indices, dtype=np.int64)
        return torch.from_numpy(self.images[idx]), torch.from_numpy(self.labels[idx])


class DeviceUpsampleLoader:
    """``DataLoader(dataset, batch_size, sampler/shuffle)`` equivalent that yields
    ``(images[B,1,H,W] f32 on device, labels[B] i64 on device)``.

    ``levels=True`` yields the resized images' uint8 levels instead of the ToTensor image (the
    ConvNet reads them as ``levels / 255``, models/convnet.py ``to_image``; its fused plan never
    materialises the fp32 image).

    On the GPU the whole 28x28 dataset lives in device memory (60 000 x 784 B = 47 MB of the
    288 GB) and each epoch's sample order is gathered into it once (one kernel per epoch), so a
    step's batch is a view of that buffer: no per-step host indexing, pinning or H2D copy -- the
    step's only input work is the upsample kernel, queued without waiting on the host.  On the
    CPU batches are gathered per step as the reference's DataLoader does."""

    def __init__(self, dataset: SyntheticMNIST, batch_size: int, image_shape, device, sampler=None,
                 shuffle: bool = False, seed: int = 0, drop_last: bool = False, levels: bool = False,
                 moments: bool = False):
        self.levels = levels
        # levels on the GPU: the upsample also forms the batch's x autocorrelation partials and
        # attaches them for the fused ConvNet plan's BN1 statistics (ops.functional.upsample_levels_moments)
        self.moments = moments and levels
        self.dataset, self.batch_size = dataset, batch_size
        self.H, self.W = image_shape
        self.device = torch.device(device)
        self.sampler, self.shuffle, self.seed, self.drop_last = sampler, shuffle, seed, drop_last
        self.epoch = 0

    def set_epoch(self, epoch: int):
        self.epoch = epoch
        if self.sampler is not None and hasattr(self.sampler, "set_epoch"):
            self.sampler.set_epoch(epoch)

    def _indices(self):
        if self.sampler is not None:
            return list(iter(self.sampler))
        n = len(self.dataset)
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            return torch.randperm(n, generator=g).tolist()
        return list(range(n))

    def __len__(self) -> int:
        n = len(self.sampler) if self.sampler is not None else len(self.dataset)
        return n // self.batch_size if self.drop_last else math.ceil(n / self.batch_size)

    def _resident(self):
        """The dataset's images and labels in device memory (uploaded once)."""
        r = getattr(self, "_dev", None)
        if r is None:
            imgs = torch.from_numpy(np.ascontiguousarray(self.dataset.images)).to(self.device)
            labs = torch.from_numpy(np.ascontiguousarray(self.dataset.labels)).to(self.device)
            r = self._dev = (imgs, labs)
        return r

    def __iter__(self):
        idx = self._indices()
        if self.device.type == "cuda":
            imgs, labs = self._resident()
            order = torch.tensor(idx, dtype=torch.int64).to(self.device, non_blocking=False)
            ep_src = imgs.index_select(0, order)  # this epoch's order, one gather
            ep_lab = labs.index_select(0, order)
            for s in range(0, len(idx), self.batch_size):
                e = min(len(idx), s + self.batch_size)
                if self.drop_last and e - s < self.batch_size:
                    break
                if self.moments:
                    from ..models import convnet_fused

                    x, part = TF.upsample_levels_moments(ep_src[s:e], self.H, self.W)
                    if part is not None:
                        convnet_fused.attach_input_stats(x, (part, None))
                    yield x, ep_lab[s:e]
                    continue
                yield TF.upsample_bilinear_u8(ep_src[s:e], self.H, self.W, levels=self.levels), ep_lab[s:e]
            return
        for s in range(0, len(idx), self.batch_size):
            b = idx[s: s + self.batch_size]
            if self.drop_last and len(b) < self.batch_size:
                break
            src, lab = self.dataset.batch(b)
            yield TF.upsample_bilinear_u8(src, self.H, self.W, levels=self.levels), lab


def synthetic_batch(batch_size: int, image_shape, device, seed: int = 0, num_classes: int = 10,
                    src: Optional[torch.Tensor] = None):
    """A fixed random batch (28x28 uint8 sources upscaled on device) — bench input."""
    g = torch.Generator()
    g.manual_seed(seed)
    if src is None:
        src = torch.randint(0, 256, (batch_size, 28, 28), generator=g, dtype=torch.uint8)
    labels = torch.randint(0, num_classes, (batch_size,), generator=g, dtype=torch.int64)
    src = src.to(device)
    return src, labels.to(device)
