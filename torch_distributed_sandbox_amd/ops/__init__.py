"""Native (gfx950 HIP) ops: functional API, nn.Module front-ends and the SGD optimizer."""
from . import functional, grad_sink
from .modules import BatchNorm2d, Conv2d, CrossEntropyLoss, Linear, MaxPool2d, ReLU
from .optim import SGD

__all__ = ["functional", "grad_sink", "Conv2d", "BatchNorm2d", "ReLU", "MaxPool2d", "Linear", "CrossEntropyLoss",
           "SGD"]
