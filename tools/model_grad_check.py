"""Model vs fp64 reference (tests/test_model_gpu.py setup) reporting EVERY parameter's relative
gradient error per step (the test stops at the first).  Env switches pass through, so the
(kernel variant A/B switches were removed; a -DTDS_DIAG build keeps the timing-only conv2 variants)
Usage: python tools/model_grad_check.py [H] [B] [steps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

from tests.test_model_gpu import RefConvNet, near_tie_windows  # noqa: E402


def main():
    from torch_distributed_sandbox_amd.models import ConvNet, fc_in_features
    from torch_distributed_sandbox_amd.ops import SGD, CrossEntropyLoss
    H = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    gpu = torch.device("cuda", 0)
    torch.manual_seed(0)
    ours = ConvNet(image_shape=(H, H), mode="auto")
    ref = RefConvNet(fc_in_features((H, H))).double()
    ref.load_state_dict({k: v.double() if v.is_floating_point() else v for k, v in ours.state_dict().items()})
    ours = ours.to(gpu)
    opt = SGD(ours.parameters(), 0.05)
    ropt = torch.optim.SGD(ref.parameters(), 0.05)
    crit = CrossEntropyLoss()
    pool_in = []
    for pool in (ref.layer1[3], ref.layer2[3]):
        pool.register_forward_hook(lambda mod, inp, out: pool_in.append(inp[0].detach()))
    env = {k: v for k, v in os.environ.items() if k.startswith("TDS_")}
    resync = os.environ.get("RESYNC", "1") == "1"  # RESYNC=0: free-running trajectories
    for s in range(steps):
        if resync:
            with torch.no_grad():
                for p, q in zip(ours.parameters(), ref.parameters()):
                    q.copy_(p.detach().double().cpu())
        x = torch.rand(B, 1, H, H, device=gpu)
        y = torch.randint(0, 10, (B,), device=gpu)
        loss = crit(ours(x), y)
        opt.zero_grad()
        loss.backward()
        pool_in.clear()
        rloss = nn.functional.cross_entropy(ref(x.double().cpu()), y.cpu())
        ties = {f"ties{t:.0e}": [near_tie_windows(a, t) for a in pool_in] for t in (1e-5, 1e-6, 1e-7)}
        ropt.zero_grad()
        rloss.backward()
        rp = dict(ref.named_parameters())
        errs = {}
        for n, p in ours.named_parameters():
            g, rg = p.grad.double().cpu(), rp[n].grad
            errs[n] = float((g - rg).norm() / rg.norm().clamp_min(1e-30))
        print({"env": env, "H": H, "B": B, "step": s, "dloss": abs(loss.item() - rloss.item()), **ties,
               **{k: f"{v:.2e}" for k, v in errs.items()}}, flush=True)
        opt.step()
        ropt.step()


if __name__ == "__main__":
    main()
