"""Per-shape implicit-GEMM timing of one eager bf16 training step (bench config).

    python tools/gemm_breakdown.py [batch] [size]

Prints, per (op, M, N, K): launches, total ms, TFLOP/s, share of GEMM time.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import cosnet_amd as C
from cosnet_amd import ops
from cosnet_amd.init_recipe import recipe_state_dict, synthetic_inputs
from cosnet_amd.optim import SGD, reference_param_groups
from cosnet_amd.train_step import TrainStep


def main():
    b = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    s = int(sys.argv[2]) if len(sys.argv) > 2 else 473
    dev = torch.device("cuda:0")
    m = C.build_model(torch.bfloat16)
    m.load_state_dict(recipe_state_dict(m.state_dict()))
    m.encoder.main_classifier.requires_grad_(False)
    m = m.to(dev).train()
    g0, g1 = reference_param_groups(m)
    opt = SGD([g0, g1], [1e-6, 1e-5])
    st = TrainStep(m, opt, b, s, graphed=False)
    st.load(*[t.to(dev) for t in synthetic_inputs(b, s, s, seed=1)])
    st.capture(warmup=2)
    torch.cuda.synchronize()
    prof = ops.GemmProfile()
    m.concurrent_encoders = False        # serialized kernels: events time one launch each
    torch.cuda._sleep(int(0.4 * 2.0e9))  # device busy while the host queues the step
    with prof:
        st.eager([1e-6, 1e-5])
    torch.cuda.synchronize()
    tags = prof.by_tag()
    tot = sum(v[2] for v in tags.values())
    fl = sum(v[1] for v in tags.values())
    print("GEMM total %.2f ms, %.1f TFLOP, %.0f TFLOP/s, %d launches" % (
        tot * 1e3, fl / 1e12, fl / tot / 1e12, sum(v[0] for v in tags.values())))
    agg = {}
    for (op, M, N, K), (n, f, t) in tags.items():
        a = agg.setdefault(op, [0, 0.0, 0.0])
        a[0] += n
        a[1] += f
        a[2] += t
    for op, (n, f, t) in sorted(agg.items(), key=lambda kv: -kv[1][2]):
        print("  %-8s %4d launches %8.2f ms %6.0f TFLOP/s %5.1f%%" % (op, n, t * 1e3, f / t / 1e12, 100 * t / tot))
    print("%-8s %7s %6s %6s %4s %8s %7s %6s" % ("op", "M", "N", "K", "n", "ms", "TF/s", "%"))
    for (op, M, N, K), (n, f, t) in sorted(tags.items(), key=lambda kv: -kv[1][2]):
        print("%-8s %7d %6d %6d %4d %8.3f %7.0f %6.2f" % (op, M, N, K, n, t * 1e3, f / t / 1e12, 100 * t / tot))


if __name__ == "__main__":
    main()
