"""Does a kernel trace survive CU-masked streams?  (`rocprofv3 --kernel-trace` over
bench.py --reserve-cus 32 segfaulted once.)  Creates the compute / comm / side streams of the CU
split (utils/streams.py), launches package kernels and a torch kernel on each, synchronizes,
prints one line.  Run it bare and under rocprofv3 with PYTHONFAULTHANDLER=1: a crash then names
the Python frame (stream creation, ExternalStream wrap, or the first launch)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import faulthandler  # noqa: E402

import torch  # noqa: E402

faulthandler.enable()


def main():
    from torch_distributed_sandbox_amd import _ext
    from torch_distributed_sandbox_amd.ops import functional as TF
    from torch_distributed_sandbox_amd.utils import streams

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ops = _ext.ops()
    src = torch.randint(0, 256, (2, 28, 28), dtype=torch.uint8, device=dev)
    print("stage: masked compute stream", flush=True)
    comp = streams.reserve_cus_for_comm(32, dev)
    print("stage: comm stream", flush=True)
    comm = streams.comm_stream(dev)
    print("stage: side stream", flush=True)
    side = streams.side_stream(dev)
    for name, st in (("compute", comp), ("comm", comm), ("side", side)):
        print(f"stage: launch on {name}", flush=True)
        with torch.cuda.stream(st):
            x = TF.upsample_bilinear_u8(src, 256, 256)
            y = (x * 2.0).sum()
        st.synchronize()
        print(f"  {name}: ok ({float(y):.3f})", flush=True)
    ops.set_cu_reserve(0)
    print("masked stream probe ok", flush=True)


if __name__ == "__main__":
    main()
