"""nn.Module front-ends for the native ops.

Parameter/buffer names and init match ``torch.nn`` exactly (``weight``,
``bias``, ``running_mean``, ``running_var``, ``num_batches_tracked``) so a
state_dict of the reference ConvNet (mnist_onegpu.py:11-31) loads unchanged.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from . import functional as TF


class Conv2d(nn.Module):
    """Stride-1 'same' convolution (``nn.Conv2d(cin, cout, k, stride=1, padding=(k-1)//2)``)."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, bias=True, device=None,
                 dtype=None):
        super().__init__()
        if stride != 1:
            raise ValueError("tds Conv2d supports stride=1 only (the reference uses stride=1)")
        if 2 * padding != kernel_size - 1:
            raise ValueError("tds Conv2d supports 'same' padding only (padding=(k-1)//2)")
        fk = {"device": device, "dtype": dtype}
        self.in_channels, self.out_channels = in_channels, out_channels
        self.kernel_size, self.stride, self.padding = (kernel_size, kernel_size), (1, 1), (padding, padding)
        self.weight = nn.Parameter(torch.empty(out_channels, in_channels, kernel_size, kernel_size, **fk))
        self.bias = nn.Parameter(torch.empty(out_channels, **fk)) if bias else None
        self.reset_parameters()

    def reset_parameters(self):
        # identical to nn.Conv2d.reset_parameters (kaiming_uniform a=sqrt(5))
        nn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        if self.bias is not None:
            fan_in = self.weight.shape[1] * self.weight.shape[2] * self.weight.shape[3]
            bound = 1 / math.sqrt(fan_in) if fan_in > 0 else 0
            nn.init.uniform_(self.bias, -bound, bound)

    def forward(self, x):
        return TF.conv2d(x, self.weight, self.bias, self.padding[0])

    def extra_repr(self):
        return f"{self.in_channels}, {self.out_channels}, kernel_size={self.kernel_size}, padding={self.padding}"


class BatchNorm2d(nn.Module):
    def __init__(self, num_features, eps=1e-5, momentum=0.1, affine=True, track_running_stats=True, device=None,
                 dtype=None):
        super().__init__()
        fk = {"device": device, "dtype": dtype}
        self.num_features, self.eps, self.momentum = num_features, eps, momentum
        self.affine, self.track_running_stats = affine, track_running_stats
        if affine:
            self.weight = nn.Parameter(torch.ones(num_features, **fk))
            self.bias = nn.Parameter(torch.zeros(num_features, **fk))
        else:
            self.register_parameter("weight", None)
            self.register_parameter("bias", None)
        if track_running_stats:
            self.register_buffer("running_mean", torch.zeros(num_features, **fk))
            self.register_buffer("running_var", torch.ones(num_features, **fk))
            self.register_buffer("num_batches_tracked", torch.tensor(0, dtype=torch.long,
                                                                     device=device))
        else:
            self.register_buffer("running_mean", None)
            self.register_buffer("running_var", None)
            self.register_buffer("num_batches_tracked", None)
        self.fuse_relu = False  # set by ConvNet when followed by ReLU

    def forward(self, x):
        use_batch = self.training or not self.track_running_stats
        return TF.batch_norm(
            x, self.running_mean if self.track_running_stats else None,
            self.running_var if self.track_running_stats else None, self.weight, self.bias, use_batch,
            self.momentum, self.eps, self.num_batches_tracked if (self.training and self.track_running_stats) else None,
            fuse_relu=self.fuse_relu,
        )

    def extra_repr(self):
        return f"{self.num_features}, eps={self.eps}, momentum={self.momentum}, affine={self.affine}"


class ReLU(nn.Module):
    def __init__(self, inplace: bool = False):
        super().__init__()
        self.inplace = inplace

    def forward(self, x):
        return TF.relu(x)


class MaxPool2d(nn.Module):
    def __init__(self, kernel_size=2, stride=2):
        super().__init__()
        if kernel_size != 2 or (stride or kernel_size) != 2:
            raise ValueError("tds MaxPool2d supports kernel_size=2, stride=2 (the reference configuration)")
        self.kernel_size, self.stride = 2, 2

    def forward(self, x):
        return TF.max_pool2x2(x)

    def extra_repr(self):
        return "kernel_size=2, stride=2"


class Linear(nn.Module):
    def __init__(self, in_features, out_features, bias=True, device=None, dtype=None):
        super().__init__()
        fk = {"device": device, "dtype": dtype}
        self.in_features, self.out_features = in_features, out_features
        self.weight = nn.Parameter(torch.empty(out_features, in_features, **fk))
        self.bias = nn.Parameter(torch.empty(out_features, **fk)) if bias else None
        self.reset_parameters()

    def reset_parameters(self):
        # nn.Linear.reset_parameters: kaiming_uniform(a=sqrt(5)) == U(-1/sqrt(fan_in), 1/sqrt(fan_in))
        bound = 1.0 / math.sqrt(self.in_features) if self.in_features > 0 else 0.0
        with torch.no_grad():
            self.weight.uniform_(-bound, bound)
            if self.bias is not None:
                self.bias.uniform_(-bound, bound)

    def forward(self, x):
        return TF.linear(x, self.weight, self.bias)

    def extra_repr(self):
        return f"in_features={self.in_features}, out_features={self.out_features}, bias={self.bias is not None}"


class CrossEntropyLoss(nn.Module):
    def __init__(self, ignore_index: int = -100, label_smoothing: float = 0.0, reduction: str = "mean"):
        super().__init__()
        if reduction != "mean":
            raise ValueError("tds CrossEntropyLoss implements reduction='mean' (the reference default)")
        self.ignore_index, self.label_smoothing = ignore_index, label_smoothing

    def forward(self, logits, labels):
        return TF.cross_entropy(logits, labels, self.ignore_index, self.label_smoothing)
