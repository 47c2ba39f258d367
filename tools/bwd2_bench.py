"""Run only the fused conv2 backward (current default version) N times at the bench shape:
a small target for rocprofv3 --pmc passes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def pack_hilo(p):
    hi = p.to(torch.bfloat16)
    lo = (p - hi.float()).to(torch.bfloat16)
    return torch.cat([hi, lo], dim=-1).contiguous().view(torch.float32)


def main():
    import torch_distributed_sandbox_amd as tds
    ops = tds._ext.ops()
    dev = torch.device("cuda", 0)
    B, P = 5, int(os.environ.get("P", 1500))
    Q = P // 2
    torch.manual_seed(0)
    y2 = torch.randn(B, P, P, 32, device=dev)
    g2m = torch.randn(B, 32, Q, Q, device=dev)
    aff2 = torch.cat([torch.rand(32, device=dev) + 0.5, torch.randn(32, device=dev)])
    kbuf = torch.randn(96, device=dev) * 0.01
    p1 = pack_hilo(torch.relu(torch.randn(B, P, P, 16, device=dev)))
    w2 = torch.randn(32, 16, 5, 5, device=dev) * 0.05
    wp, wd = ops.conv2_pack(w2)
    which = sys.argv[1] if len(sys.argv) > 1 else "bwd"
    for _ in range(int(os.environ.get("N", 5))):
        if which == "bwd":
            ops.fused_conv2_backward_y2(y2, g2m, aff2, kbuf, p1, wd, 1.0)
        else:
            ops.fused_conv2_forward(p1, wp, w2.new_zeros(32))
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
