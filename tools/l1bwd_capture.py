"""Runs the model-vs-reference comparison (H=128, B=2, as tests/test_model_gpu.py) and, at each
layer-1 backward, compares the MFMA and sparse kernels on the model's own inputs; saves the
step-1 inputs to gpurun_out/l1cap.pt (weights_only-loadable tensors)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import torch_distributed_sandbox_amd._ext as ext  # noqa: E402

_real_ops = ext.ops
calls = []


class _Proxy:
    def __getattr__(self, name):
        real = getattr(_real_ops(), name)
        if name != "fused_l1_backward":
            return real

        def wrapped(*a):
            outs = {}
            for ver in ("1", "0"):
                os.environ["TDS_L1_BWD"] = ver
                outs[ver] = [t.clone() for t in real(*a)]
            os.environ.pop("TDS_L1_BWD")
            s, m = outs["1"], outs["0"]
            print({"call": len(calls), "dw1_rel": float((m[0] - s[0]).norm() / s[0].norm()),
                   "db1": float((m[1] - s[1]).abs().max()), "dg_rel": float((m[2] - s[2]).norm() / s[2].norm()),
                   "dbe_rel": float((m[3] - s[3]).norm() / s[3].norm())}, flush=True)
            calls.append({k: v.detach().cpu() if torch.is_tensor(v) else torch.tensor(v)
                          for k, v in zip(("dp1", "x", "p1", "idx1", "w1", "b1", "g1", "stats1", "gram", "scale"), a)})
            return tuple(m)
        return wrapped


ext.ops = lambda: _Proxy()
from tests.test_model_gpu import _compare  # noqa: E402

try:
    _compare("auto", torch.device("cuda", 0), H=128, B=2)
    print("compare passed")
except AssertionError as e:
    print("compare failed:", e)
os.makedirs("gpurun_out", exist_ok=True)
torch.save(calls, "gpurun_out/l1cap.pt")
