"""A/B of the co-attention kernel variants (cn_coatt_force_variant) at the bench shapes:
the no-grad forward (configs[3]: 5 pairs; and 4 pairs), the training forward with LSE (4 pairs)
the PV and dVa_t backward kernels (4 / 8 pairs), 60 x 60 features, C = 256, bf16.  Device time per call from
a HIP graph of R calls (no host gaps); TFLOP/s counts the executed S and PV products (2 x 2 HW^2 C
per pair and direction).

    python tools/coatt_variant_ab.py [variants=1,5] [pairs=5,4] [--nograd-only]   (or 1+5 / 8+4)
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cosnet_amd import _native as nv   # noqa: E402
from cosnet_amd import ops             # noqa: E402

R = 20


def timed(fn):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(R):
            fn()
    ts = []
    for _ in range(4):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts = sorted(ts[1:])
    return ts[len(ts) // 2] / R * 1e3   # us per call


def main():
    args = [x for x in sys.argv[1:] if not x.startswith("--")]
    nograd_only = "--nograd-only" in sys.argv
    # lists comma- or plus-separated (tools/gpu_pass.sh py: steps turn commas into spaces)
    variants = [int(x) for x in (args[0] if args else "1,5").replace("+", ",").split(",")]
    pairs = [int(x) for x in (args[1] if len(args) > 1 else "5,4").replace("+", ",").split(",")]
    lib = nv.load()
    dev = torch.device("cuda:0")
    hw, c = 3600, 256
    out = []
    for n in pairs:
        g = torch.Generator().manual_seed(n)
        vat, va, vb, dzb = [(torch.randn((n * hw, c), generator=g) * 0.7).to(torch.bfloat16).to(dev)
                            for _ in range(4)]
        za, zb = torch.empty_like(va), torch.empty_like(va)
        la = torch.empty((n, ops.hw_pad(hw)), dtype=torch.float32, device=dev)
        lb = torch.empty_like(la)
        pv = torch.zeros_like(va)
        ops.coatt_flash_fwd(vat, va, vb, n, hw, za, zb, la, lb)
        flop_dir = 2 * 2.0 * n * hw * hw * c
        for v in variants:
            old = lib.cn_coatt_force_variant(v)
            if old == -1:
                continue
            try:
                nws = int(nv.query("cn_coatt_fused_workspace_bytes", n, hw, 1))
                ws = torch.empty((max(nws, 4) // 4,), dtype=torch.float32, device=dev)
                row = {"variant": v, "n": n,
                       "nograd_fwd_us": timed(lambda: ops.coatt_fused(vat, va, vb, n, hw, za, zb))}
                if n in (4, 8) and not nograd_only:
                    row["train_fwd_us"] = timed(lambda: ops.coatt_flash_fwd(vat, va, vb, n, hw, za, zb, la, lb))
                    row["pv_us"] = timed(lambda: nv.call(
                        "cn_coatt_flash_pv_ws", vat.data_ptr(), 256, vb.data_ptr(), 256, dzb.data_ptr(), 256,
                        lb.data_ptr(), n, hw, 256, pv.data_ptr(), 256, 0, ws.data_ptr(), nws, nv.stream()))
                    row["pv_tflops"] = flop_dir / row["pv_us"] / 1e6
                    # the dVa_t backward kernel (both gradient terms, with its two row-dot passes)
                    row["dvat_us"] = timed(lambda: ops.coatt_flash_bwd(
                        vat, va, vb, None, za, zb, la, lb, dzb, dzb, n, hw))
                    row["train_fwd_tflops"] = 2 * flop_dir / row["train_fwd_us"] / 1e6
                row["nograd_fwd_tflops"] = 2 * flop_dir / row["nograd_fwd_us"] / 1e6
            finally:
                lib.cn_coatt_force_variant(old)
            out.append(row)
            print(json.dumps({k: (round(x, 2) if isinstance(x, float) else x) for k, x in row.items()}), flush=True)


if __name__ == "__main__":
    main()
