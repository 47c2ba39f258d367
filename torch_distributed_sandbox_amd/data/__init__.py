"""Synthetic MNIST-like data with on-device upscaling."""
from .synthetic import MNIST_TRAIN_SIZE, DeviceUpsampleLoader, SyntheticMNIST, synthetic_batch

__all__ = ["SyntheticMNIST", "DeviceUpsampleLoader", "synthetic_batch", "MNIST_TRAIN_SIZE"]
