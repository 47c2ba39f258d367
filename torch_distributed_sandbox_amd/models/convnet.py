"""The reference's ConvNet (mnist_onegpu.py:11-31 == mnist_distributed.py:25-45).

    layer1: Conv2d(1,16,5,1,2) -> BatchNorm2d(16) -> ReLU -> MaxPool2d(2,2)
    layer2: Conv2d(16,32,5,1,2) -> BatchNorm2d(32) -> ReLU -> MaxPool2d(2,2)
    fc    : Linear(32*(H//4)*(W//4), num_classes)

Differences from the reference, by design:

* ``fc.in_features`` is derived analytically from ``image_shape`` instead of a
  ``LazyLinear`` materialised by a 65-GFLOP dummy forward on the CPU
  (mnist_onegpu.py:38-39).
* Module and parameter names are identical (``layer1.0.weight`` ...
  ``fc.bias``), so reference state_dicts load as-is.
* ``forward`` picks an execution plan: on GPU in training mode the fused
  gfx950 plan (``models/convnet_fused.py``) runs the whole network as five
  fused kernels per direction; otherwise the layer-by-layer native ops run
  (``mode='layers'``), and on CPU the PyTorch reference ops.
* ``forward`` also takes a uint8 batch: the resized images' levels before the
  reference's ``ToTensor`` (mnist_onegpu.py:50-52), read as ``levels / 255``
  (``to_image``).  The fused plan folds that scale into conv1 and its batch
  statistics, so the fp32 image (4x the bytes) is never written or read; the
  other plans convert first.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ..ops import modules as M

IMAGE_SHAPE = (3000, 3000)
LEVEL_SCALE = 1.0 / 255.0  # fp32(1/255): the scale ToTensor and the upsample kernel apply to uint8 levels


def to_image(x: torch.Tensor) -> torch.Tensor:
    """fp32 image of a uint8 level batch (x * fp32(1/255), as the upsample kernel scales);
    fp32 batches pass through."""
    if x.dtype == torch.uint8:
        return x.float().mul_(torch.tensor(LEVEL_SCALE, dtype=torch.float32).item())
    return x


def fc_in_features(image_shape, channels: int = 32) -> int:
    h, w = image_shape
    return channels * ((h // 2) // 2) * ((w // 2) // 2)


class ConvNet(nn.Module):
    def __init__(self, num_classes: int = 10, image_shape=IMAGE_SHAPE, device=None, mode: str = "auto"):
        super().__init__()
        self.image_shape = tuple(image_shape)
        self.layer1 = nn.Sequential(
            M.Conv2d(1, 16, kernel_size=5, stride=1, padding=2, device=device),
            M.BatchNorm2d(16, device=device),
            M.ReLU(),
            M.MaxPool2d(kernel_size=2, stride=2),
        )
        self.layer2 = nn.Sequential(
            M.Conv2d(16, 32, kernel_size=5, stride=1, padding=2, device=device),
            M.BatchNorm2d(32, device=device),
            M.ReLU(),
            M.MaxPool2d(kernel_size=2, stride=2),
        )
        self.fc = M.Linear(fc_in_features(self.image_shape), num_classes, device=device)
        if mode not in ("auto", "fused", "layers"):
            raise ValueError(f"mode must be auto|fused|layers, got {mode!r}")
        self.mode = mode

    # ------------------------------------------------------------------ plans
    def _forward_layers(self, x):
        # BN + ReLU fused into one native pass on the GPU (the ReLU module is then skipped)
        for layer in (self.layer1, self.layer2):
            conv, bn, act, pool = layer
            x = conv(x)
            if x.is_cuda:
                bn.fuse_relu = True
                x = bn(x)
            else:
                bn.fuse_relu = False
                x = act(bn(x))
            x = pool(x)
        x = x.reshape(x.size(0), -1)
        return self.fc(x)

    def _use_fused(self, x) -> bool:
        if self.mode == "layers" or not x.is_cuda:
            return False
        from . import convnet_fused

        ok = convnet_fused.supported(self, x)
        if self.mode == "fused" and not ok:
            raise RuntimeError("ConvNet(mode='fused'): input/config not supported by the fused plan")
        return ok

    def forward(self, x):
        if self._use_fused(x):
            from . import convnet_fused

            return convnet_fused.forward(self, x)
        return self._forward_layers(to_image(x))
