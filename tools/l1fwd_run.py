"""Run only the layer-1 forward N times at the bench shape (rocprofv3 --pmc target)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    import torch_distributed_sandbox_amd as tds
    from torch_distributed_sandbox_amd.ops import functional as TF
    ops = tds._ext.ops()
    dev = torch.device("cuda", 0)
    B, H = 5, int(os.environ.get("H", 3000))
    torch.manual_seed(0)
    x = TF.upsample_bilinear_u8(torch.randint(0, 256, (B, 28, 28), dtype=torch.uint8, device=dev), H, H)
    w1 = torch.randn(16, 1, 5, 5, device=dev) * 0.2
    b1 = torch.randn(16, device=dev) * 0.1
    g1 = torch.rand(16, device=dev) + 0.5
    be1 = torch.randn(16, device=dev) * 0.1
    for _ in range(int(os.environ.get("N", 5))):
        ops.fused_l1_forward(x, w1, b1, g1, be1, None, None, None, 0.1, 1e-5)
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
