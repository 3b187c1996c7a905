"""bf16 vs fp8 conv forward GEMM time on the step's main shapes (+ the quantisation pass)."""
import sys
sys.path.insert(0, '.')
import torch
from cosnet_amd import ops
dev = torch.device('cuda:0')
SH = {"aspp": (8, 2048, 60, 60, 512, 3, 1, 12, 12), "l4": (8, 512, 60, 60, 512, 3, 1, 4, 4),
      "l3": (8, 256, 60, 60, 256, 3, 1, 2, 2), "l3_1x1": (8, 1024, 60, 60, 256, 1, 1, 0, 1),
      "l3b_1x1": (8, 256, 60, 60, 1024, 1, 1, 0, 1), "asppb": (8, 2560, 60, 60, 256, 3, 1, 1, 1)}


def tm(fn, reps=30):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for name, (n, cin, h, w, cout, k, s, p, d) in SH.items():
    x = torch.randn(n * h * w, cin, device=dev).to(torch.bfloat16)
    wf = (torch.randn(cout, k * k * cin, device=dev) * 0.05).to(torch.bfloat16)
    xs, ws = ops.fp8_state(dev), ops.fp8_state(dev)
    x8 = ops.fp8_quant(x, xs)
    w8 = ops.fp8_quant(wf.float(), ws)
    fl = 2.0 * n * h * w * cout * k * k * cin
    t0 = tm(lambda: ops.conv_fwd(x, n, h, w, wf, cout, k, s, p, d))
    t1 = tm(lambda: ops.conv_fwd_fp8(x8, n, h, w, w8, cout, k, s, p, d, xs, ws))
    t2 = tm(lambda: ops.fp8_quant(x, xs, ops.FP8_DELAYED, out=x8))
    print("%-8s bf16 %7.1f us (%5.0f TF/s)  fp8 %7.1f us (%5.0f TF/s)  quant %5.1f us" % (
        name, t0, fl / t0 / 1e6, t1, fl / t1 / 1e6, t2), flush=True)
