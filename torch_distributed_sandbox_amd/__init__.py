"""torch_distributed_sandbox_amd — an MI355X-native (gfx950, CDNA4) data-parallel training sandbox.

Same capability surface as AditMeh/torch-distributed-sandbox (all-reduce toy,
process-group init test, single-GPU and DDP trainers for a ConvNet on
3000x3000 MNIST), rebuilt for MI355X: hand-written HIP kernels for the hot ops
(``ops``), a DDP with flat buckets and gradient sinks over RCCL/xGMI
(``parallel``), on-device synthetic data (``data``).
"""
from . import _ext

__version__ = "0.1.0"

__all__ = ["_ext", "__version__"]
