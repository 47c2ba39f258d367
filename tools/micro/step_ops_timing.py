"""Per-op timing of the fused ConvNet step at the bench shape (3000x3000, B=5), each op run in
isolation on the tensors a real step produces (CUDA events, median of 5 rounds x N iterations).
Usage: python tools/micro/step_ops_timing.py [--iters 20] [--only conv2_bwd,...]
With TDS_SO_VARIANT=<name> it times the side build _C_<name>.so (A/B experiments)."""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import torch_distributed_sandbox_amd as tds  # noqa: E402


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(iters):
            fn()
        b.record()
        torch.cuda.synchronize()
        out.append(a.elapsed_time(b) / iters)
    return statistics.median(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--image-size", type=int, default=3000)
    ap.add_argument("--batch-size", type=int, default=5)
    ap.add_argument("--only", default="")
    ap.add_argument("--reserve-cus", type=int, default=0, help="run on a CU-masked stream (utils/streams.py)")
    a = ap.parse_args()
    ops = tds._ext.ops()
    if a.reserve_cus:
        from torch_distributed_sandbox_amd.utils.streams import reserve_cus_for_comm

        torch.cuda.set_stream(reserve_cus_for_comm(a.reserve_cus, torch.device("cuda", 0)))
    from torch_distributed_sandbox_amd.data import synthetic_batch
    from torch_distributed_sandbox_amd.models import ConvNet
    from torch_distributed_sandbox_amd.ops import functional as TF

    dev = torch.device("cuda", 0)
    H, B = a.image_size, a.batch_size
    P = H // 2
    torch.manual_seed(0)
    m = ConvNet(image_shape=(H, H), device=dev)
    c1, n1, c2, n2, fc = m.layer1[0], m.layer1[1], m.layer2[0], m.layer2[1], m.fc
    src, _ = synthetic_batch(B, (H, H), dev, seed=7)
    x = TF.upsample_bilinear_u8(src, H, H)
    with torch.no_grad():
        st = {}

        def l1f():
            st["l1"] = ops.fused_l1_forward(x, c1.weight, c1.bias, n1.weight, n1.bias, n1.running_mean,
                                            n1.running_var, n1.num_batches_tracked, 0.1, 1e-5)

        def pack():
            st["mag"] = torch.zeros(ops.mag_numel(B, P), dtype=torch.int32, device=x.device)
            st["pack"] = ops.conv2_pack(c2.weight, st["mag"])

        def c2f():
            st["c2"] = ops.fused_conv2_forward(st["l1"][0], st["pack"][0], c2.bias, n2.weight, st["mag"])

        def hf():
            y2, partial2, ya = st["c2"][:3]
            st["hf"] = ops.fused_head_forward(ya, partial2, c2.bias, n2.weight, n2.bias, n2.running_mean,
                                              n2.running_var, n2.num_batches_tracked, 0.1, 1e-5, fc.weight,
                                              fc.bias, P, None, mag=st["mag"])

        dl = torch.randn(B, 10, device=dev) * 0.1
        dw = torch.empty_like(fc.weight)

        def hb():
            _, stats2, aff2 = st["hf"]
            st["hb"] = ops.fused_head_backward(dl, st["c2"][2], stats2, aff2, c2.bias, n2.weight, fc.weight, P, dw, 1.0,
                                               True,
                                               mag=st["mag"])

        def hb_nomag():  # A/B: the same launch without the |g2m| bound (atomic max)
            _, stats2, aff2 = st["hf"]
            ops.fused_head_backward(dl, st["c2"][2], stats2, aff2, c2.bias, n2.weight, fc.weight, P, dw, 1.0, True)

        def c2b():
            y2 = st["c2"][0]
            g2m, kbuf = st["hb"][4], st["hb"][5]
            st["c2b"] = ops.fused_conv2_backward_y2(y2, st["c2"][3], g2m, st["hf"][2], kbuf, c2.bias, st["mag"], st["l1"][0],
                                                        st["pack"][1], 1.0)

        def l1b():
            p1, idx1, stats1, gram = st["l1"][:4]
            ops.fused_l1_backward(st["c2b"][0], st["mag"][44:45], x, p1, idx1, c1.weight, c1.bias, n1.weight, stats1,
                                  gram, 1.0)

        # the activation exchange's pieces (parallel/factored.py, world 1): the head forward writing X,
        # the zero-suppressed encode of that X and the update sweep over the encodings
        from torch_distributed_sandbox_amd.parallel import zs

        K = fc.weight.shape[1]
        xo = torch.empty(B, K, device=dev)
        w2c = fc.weight.detach().clone()
        meta = torch.empty(zs.meta_numel(B * K), device=dev, dtype=torch.int32)
        vals = torch.empty(B * K, device=dev)

        def hf_x():
            ops.fused_head_forward_aff(st["c2"][2], st["hf"][2], c2.bias, st["mag"], w2c, fc.bias, P, xo)

        def enc_x():
            st["nnz"] = zs.encode(xo, meta, vals)

        def dw_zs():
            ops.linear_dw_zs(dl, meta.view(1, -1), vals.view(1, -1), B, w2c, None, 1.0, False, 1e-12)

        xl = TF.upsample_bilinear_u8(src, H, H, levels=True)

        def ups():  # the bench's input op: uint8 levels
            TF.upsample_bilinear_u8(src, H, H, levels=True)

        def moments():  # the x moments' partials + border strips + reduction (levels input)
            ops.l1_input_stats(xl)

        def ups_mom():  # the input op fused with the moments' partials
            st["um"] = ops.upsample_levels_moments(src, H, H)

        def l1f_u8():  # the layer-1 forward on levels, reducing the fused op's partials (border strips in-launch)
            ops.fused_l1_forward(st["um"][0], c1.weight, c1.bias, n1.weight, n1.bias, n1.running_mean,
                                 n1.running_var, n1.num_batches_tracked, 0.1, 1e-5, st["um"][1], None)

        def l1f_u8_self():  # ... forming the moments itself (autocorrelation + in-launch border)
            ops.fused_l1_forward(xl, c1.weight, c1.bias, n1.weight, n1.bias, n1.running_mean,
                                 n1.running_var, n1.num_batches_tracked, 0.1, 1e-5, None, None)

        seq = [("ups", ups), ("moments", moments), ("ups_mom", ups_mom), ("l1_fwd_u8", l1f_u8),
               ("l1_fwd_u8_self", l1f_u8_self), ("l1_fwd", l1f), ("conv2_pack", pack), ("conv2_fwd", c2f), ("head_fwd", hf), ("head_bwd", hb),
               ("head_bwd_nomag", hb_nomag), ("conv2_bwd", c2b), ("l1_bwd", l1b),
               ("head_fwd_x", hf_x), ("zs_enc_x", enc_x), ("dw_zs", dw_zs)]
        only = set(a.only.split(",")) if a.only else None
        for name, fn in seq:
            if name in ("head_fwd_x", "zs_enc_x", "dw_zs") and only and not (
                    only & {"head_fwd_x", "zs_enc_x", "dw_zs"}):
                continue
            fn()
        only = set(a.only.split(",")) if a.only else None
        res = {}
        for name, fn in seq:
            if only and name not in only:
                continue
            res[name] = round(timeit(fn, a.iters), 4)
            print(f"{name:11s} {res[name]:.4f} ms", flush=True)
        if os.environ.get("TDS_CONV2_DIAG", "0") == "13" or int(os.environ.get("TDS_CONV2_DIAG", "0") or 0) >= 16:  # per-role barrier-wait fractions (diag build)
            c2b()
            torch.cuda.synchronize()
            clk = ops.conv2_bwd_clock_dump(ops.device_cus()).to(torch.int64) & 0xFFFFFFFF
            for name, sl in (("dgrad", slice(0, 2)), ("wgrad", slice(2, 4)), ("staging", slice(4, 8))):
                w, t = clk[:, sl, 0].sum().item(), clk[:, sl, 1].sum().item()
                print(f"clock {name:8s} waits {w / max(t, 1):.3f} of its run "
                      f"(mean run {clk[:, sl, 1].float().mean().item():.0f} cycles)", flush=True)
        print(json.dumps({"variant": os.environ.get("TDS_SO_VARIANT", ""), "ms": res,
                          "sum_ms": round(sum(res.values()), 4)}), flush=True)


if __name__ == "__main__":
    main()
