"""Allocated-memory trace of one fused ConvNet step (forward, backward, grads dropped, loss dropped)."""
import sys

import torch

sys.path.insert(0, ".")
from torch_distributed_sandbox_amd.models import ConvNet  # noqa: E402
from torch_distributed_sandbox_amd.ops import CrossEntropyLoss  # noqa: E402

H = int(sys.argv[1]) if len(sys.argv) > 1 else 24000
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1
dev = torch.device("cuda", 0)
gb = lambda: round(torch.cuda.memory_allocated(dev) / 1e9, 2)  # noqa: E731
m = ConvNet(image_shape=(H, H), device=dev, mode="fused")
print("model", gb(), flush=True)
x = torch.rand(B, 1, H, H, device=dev)
y = torch.zeros(B, dtype=torch.long, device=dev)
print("x", gb(), flush=True)
logits = m(x)
print("forward", gb(), flush=True)
loss = CrossEntropyLoss()(logits, y)
loss.backward()
torch.cuda.synchronize()
print("backward", gb(), "peak", round(torch.cuda.max_memory_allocated(dev) / 1e9, 2), flush=True)
for p in m.parameters():
    p.grad = None
print("grads dropped", gb(), flush=True)
del loss, logits
print("loss dropped", gb(), flush=True)
