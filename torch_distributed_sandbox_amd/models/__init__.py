"""Model zoo: the reference's 3000x3000 MNIST ConvNet."""
from .convnet import IMAGE_SHAPE, ConvNet, fc_in_features

__all__ = ["ConvNet", "IMAGE_SHAPE", "fc_in_features"]
