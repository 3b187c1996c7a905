"""Per-shape time and achieved HBM bandwidth of the BN passes (bf16), measured by replaying a
HIP graph of REPS launches (no host launch overhead in the number)."""
import sys

import torch

sys.path.insert(0, '.')
from cosnet_amd import ops  # noqa: E402
from cosnet_amd import _native as nv  # noqa: E402

dev = torch.device('cuda:0')
dt = torch.bfloat16
REPS = 20


def gtime(fn):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(REPS):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (5 * REPS) * 1e-3


def main():
    for kv in sys.argv[1:]:
        k, v = kv.split('=')
        nv.call("cn_bn_set_tuning", int(k), int(v))
    shapes = [(14400, 256, 2), (14400, 1024, 2), (14400, 512, 2), (56644, 64, 2), (56644, 256, 2),
              (224676, 64, 2), (14400, 2048, 2)]
    tot = {}
    for P, C, ns in shapes:
        x = torch.randn(P * ns, C, device=dev).to(dt)
        r = torch.randn(P * ns, C, device=dev).to(dt)
        bn = torch.nn.BatchNorm2d(C).to(dev)
        st = ops.bn_stats(x, bn, True, nseg=ns)
        y = ops.bn_apply(x, st, bn, act=1, nseg=ns)
        xa, ra, ya = x[:P], r[:P], y[:P]
        sta = ops.seg_of(st, 0, C)
        nb = P * ns * C * 2
        t = {
            'stats': (gtime(lambda: ops.bn_stats(x, bn, True, nseg=ns)), nb),
            'apply': (gtime(lambda: ops.bn_apply(x, st, bn, act=1, out=y, nseg=ns)), 2 * nb),
            'apply+xr': (gtime(lambda: ops.bn_apply(x, st, bn, act=1, xr=r, rstats=st, rbn=bn, out=y, nseg=ns)), 3 * nb),
            'bwd': (gtime(lambda: ops.bn_bwd(xa, ra, ya, sta, bn, act=1)), 7 * nb // ns),
            'bwd_noapply': (gtime(lambda: ops.bn_bwd(xa, ra, ya, sta, bn, act=1, want_dx=False)), 3 * nb // ns),
        }
        line = "P=%6dx%d C=%4d" % (P, ns, C)
        for k, (tt, b) in t.items():
            line += " | %s %5.1f us %5.0f GB/s" % (k, tt * 1e6, b / tt / 1e9)
            tot[k] = tot.get(k, 0) + tt
        print(line, flush=True)
    print("sum over shapes (us):", {k: round(v * 1e6, 1) for k, v in tot.items()}, flush=True)


if __name__ == "__main__":
    main()
