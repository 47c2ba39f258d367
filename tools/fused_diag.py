"""Per-parameter gradient error of the fused plan (and the exact layers plan) vs an fp64 reference."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn as nn
import torch.nn.functional as F
from torch_distributed_sandbox_amd.models import ConvNet, fc_in_features
from torch_distributed_sandbox_amd.ops import CrossEntropyLoss


class Ref(nn.Module):
    def __init__(self, inf):
        super().__init__()
        self.layer1 = nn.Sequential(nn.Conv2d(1, 16, 5, 1, 2), nn.BatchNorm2d(16), nn.ReLU(), nn.MaxPool2d(2, 2))
        self.layer2 = nn.Sequential(nn.Conv2d(16, 32, 5, 1, 2), nn.BatchNorm2d(32), nn.ReLU(), nn.MaxPool2d(2, 2))
        self.fc = nn.Linear(inf, 10)

    def forward(self, x):
        o = self.layer2(self.layer1(x))
        return self.fc(o.reshape(o.size(0), -1))


def run(mode, H, B, seed=0):
    dev = torch.device("cuda", 0)
    torch.manual_seed(seed)
    ours = ConvNet(image_shape=(H, H), mode=mode)
    ref = Ref(fc_in_features((H, H))).double()
    ref.load_state_dict({k: v.double() if v.is_floating_point() else v for k, v in ours.state_dict().items()})
    ours = ours.to(dev)
    x = torch.rand(B, 1, H, H, device=dev)
    y = torch.randint(0, 10, (B,), device=dev)
    loss = CrossEntropyLoss()(ours(x), y)
    loss.backward()
    rl = F.cross_entropy(ref(x.double().cpu()), y.cpu())
    rl.backward()
    rp = dict(ref.named_parameters())
    out = [f"{mode:6s} H={H:4d} B={B} loss {loss.item():.6f} ref {rl.item():.6f}"]
    for n, p in ours.named_parameters():
        g, rg = p.grad.double().cpu(), rp[n].grad
        e = (g - rg).abs().max().item()
        s = rg.abs().max().item()
        out.append(f"   {n:18s} rel {e / max(s, 1e-30):.2e}  (err {e:.2e} scale {s:.2e})")
    print("\n".join(out), flush=True)


if __name__ == "__main__":
    for H in (64, 128, 256):
        for mode in ("fused", "layers"):
            run(mode, H, 2)
