"""Single-GPU ConvNet trainer on 3000x3000 (synthetic) MNIST — MI355X-native.

Reference: mnist_onegpu.py (train(0, args) without spawn, bs=5, SGD lr=1e-4).
Usage:  python mnist_onegpu.py --epochs 2 [--max-steps N] [--image-size 3000] [--batch-size 5]
"""
import argparse

from torch_distributed_sandbox_amd.trainer import add_common_args, train


def main(argv=None):
    parser = add_common_args(argparse.ArgumentParser(description=__doc__.split("\n")[0]))
    args = parser.parse_args(argv)
    return train(0, args, distributed=False)


if __name__ == "__main__":
    main()
