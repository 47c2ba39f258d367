"""Where the workgroups of a (CU-masked) stream land: XCC id and CU (HW_ID bits 8-15) per
workgroup, summarised per XCC.  Used to check hipExtStreamCreateWithCUMask's bit numbering
(utils/streams.py, csrc/kernels/cu_budget.hip) on MI355X.

    python tools/micro/cu_probe.py
"""
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from torch_distributed_sandbox_amd import _ext  # noqa: E402


def summary(out):
    per = collections.defaultdict(set)
    wgs = collections.Counter()
    for xcc, hw in out.tolist():
        key = (hw >> 8) & 0xFF
        per[xcc].add(key)
        wgs[xcc] += 1
    return {x: (len(per[x]), wgs[x]) for x in sorted(per)}


def main():
    ops = _ext.ops()
    dev = torch.device("cuda", 0)
    like = torch.empty(1, device=dev)
    n = ops.device_cus()
    print("device CUs", n)
    configs = [("unmasked", None)]
    for r in (16, 32):
        for striped in (True, False):
            configs.append((f"reserve{r}_{'striped' if striped else 'blocked'}", (r, striped)))
    for name, cfg in configs:
        if cfg is None:
            s = torch.cuda.current_stream(dev)
        else:
            s = torch.cuda.ExternalStream(ops.cu_masked_stream(0, cfg[0], cfg[1]), device=dev)
        with torch.cuda.stream(s):
            out = ops.cu_probe(like, 200, 2048)
        torch.cuda.synchronize()
        sm = summary(out.cpu())
        tot = sum(v[0] for v in sm.values())
        print(f"{name:24s} CUs used {tot:4d}  per XCC (CUs, WGs): {sm}", flush=True)


if __name__ == "__main__":
    main()
