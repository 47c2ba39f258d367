"""Reference-stack comparison: the reference ConvNet in eager PyTorch-ROCm (MIOpen convs,
ATen BN/pool/linear, torch.optim.SGD) at the same config as bench.py.  Prints one JSON line.
This is what the reference code would run at on MI355X (minus its CPU-bound PIL input pipeline)."""
import argparse
import json
import time

import torch
import torch.nn as nn


class ConvNet(nn.Module):
    def __init__(self, in_features, num_classes=10):
        super().__init__()
        self.layer1 = nn.Sequential(nn.Conv2d(1, 16, 5, 1, 2), nn.BatchNorm2d(16), nn.ReLU(), nn.MaxPool2d(2, 2))
        self.layer2 = nn.Sequential(nn.Conv2d(16, 32, 5, 1, 2), nn.BatchNorm2d(32), nn.ReLU(), nn.MaxPool2d(2, 2))
        self.fc = nn.Linear(in_features, num_classes)

    def forward(self, x):
        out = self.layer2(self.layer1(x))
        return self.fc(out.reshape(out.size(0), -1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--image-size", type=int, default=3000)
    ap.add_argument("--batch-size", type=int, default=5)
    ap.add_argument("--tf32", action="store_true")
    a = ap.parse_args()
    torch.backends.cudnn.allow_tf32 = a.tf32
    dev = torch.device("cuda", 0)
    H = a.image_size
    torch.manual_seed(0)
    m = ConvNet(32 * (H // 4) ** 2).to(dev)
    crit = nn.CrossEntropyLoss()
    opt = torch.optim.SGD(m.parameters(), 1e-4)
    x = torch.rand(a.batch_size, 1, H, H, device=dev)
    y = torch.randint(0, 10, (a.batch_size,), device=dev)

    def step():
        loss = crit(m(x), y)
        opt.zero_grad()
        loss.backward()
        opt.step()
        return loss

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"stack": "pytorch-eager-rocm", "images_per_sec": a.batch_size * a.steps / dt,
                      "ms_per_step": 1e3 * dt / a.steps, "image_size": H, "batch": a.batch_size,
                      "peak_mem_gb": torch.cuda.max_memory_allocated(dev) / 1e9}))


if __name__ == "__main__":
    main()
