"""Achieved HBM bandwidth of the BN kernels on the step's shapes (bf16)."""
import sys, torch
sys.path.insert(0, '.')
from cosnet_amd import ops
dev = torch.device('cuda:0')
dt = torch.bfloat16
def bench(fn, reps=20):
    fn(); torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3
for P, C in [(14400, 256), (14400, 1024), (14400, 512), (56644, 64), (56644, 256), (224676, 64), (14400, 2048)]:
    x = torch.randn(P, C, device=dev).to(dt)
    r = torch.randn(P, C, device=dev).to(dt)
    bn = torch.nn.BatchNorm2d(C).to(dev)
    st = ops.bn_stats(x, bn, True)
    y = ops.bn_apply(x, st, bn, act=1)
    nb = P * C * 2
    t_st = bench(lambda: ops.bn_stats(x, bn, True))
    t_ap = bench(lambda: ops.bn_apply(x, st, bn, act=1, out=y))
    t_apr = bench(lambda: ops.bn_apply(x, st, bn, act=1, res=r, out=y))
    t_bw = bench(lambda: ops.bn_bwd(x, r, y, st, bn, act=1))
    print("P=%6d C=%4d %6.1f MB | stats %6.1f us %5.0f GB/s | apply %6.1f us %5.0f GB/s | apply+res %6.1f us %5.0f GB/s | bwd %6.1f us %5.0f GB/s" % (
        P, C, nb / 1e6, t_st * 1e6, nb / t_st / 1e9, t_ap * 1e6, 2 * nb / t_ap / 1e9, t_apr * 1e6, 3 * nb / t_apr / 1e9,
        t_bw * 1e6, 7 * nb / t_bw / 1e9), flush=True)
