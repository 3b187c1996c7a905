"""Warm vs cold-cache per-launch time of the implicit GEMM on the step's hot conv shapes, per
tile configuration.  'warm' replays one operand set (L2 / MALL resident, what gemm_lab and the
config sweep measure); 'cold' cycles through enough distinct operand sets (> 600 MB) that every
launch reads its operands from HBM, as in the training step where each conv reads a tensor the
previous kernel wrote and its weights once.
usage: python tools/gemm_cold.py [filter] [configs, e.g. 11,13,14]"""
import sys

import torch

sys.path.insert(0, '.')
from cosnet_amd import _native as nv  # noqa: E402
from cosnet_amd import ops  # noqa: E402

dev = torch.device('cuda:0')
dt = torch.bfloat16
# name, op, n, cin, h, w, cout, k, pad, dil   (backward ops at the frame batch n=4)
SHAPES = [
    ("l3_3x3_d2 fwd", "fwd", 8, 256, 60, 60, 256, 3, 2, 2),
    ("l3_3x3_d2 dgrad", "dgrad", 4, 256, 60, 60, 256, 3, 2, 2),
    ("l3_1x1_1024to256 fwd", "fwd", 8, 1024, 60, 60, 256, 1, 0, 1),
    ("l3_1x1_1024to256 dgrad", "dgrad", 4, 1024, 60, 60, 256, 1, 0, 1),
    ("l3_1x1_256to1024 fwd", "fwd", 8, 256, 60, 60, 1024, 1, 0, 1),
    ("l3_1x1_256to1024 dgrad", "dgrad", 4, 256, 60, 60, 1024, 1, 0, 1),
    ("l4_3x3_512_d4 fwd", "fwd", 8, 512, 60, 60, 512, 3, 4, 4),
    ("l4_3x3_512_d4 dgrad", "dgrad", 4, 512, 60, 60, 512, 3, 4, 4),
    ("aspp_3x3_d12 fwd", "fwd", 8, 2048, 60, 60, 512, 3, 12, 12),
]


def gtime_sets(fns, reps=3):
    for f in fns:
        f()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for f in fns:
            f()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            for f in fns:
                f()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (3 * reps * len(fns)) * 1e-3


def main():
    flt = sys.argv[1] if len(sys.argv) > 1 and sys.argv[1] != "all" else ""
    cfgs = [int(c) for a in sys.argv[2:] for c in a.split(",")] if len(sys.argv) > 2 else [-1, 11, 13, 14, 7, 2]
    for (name, op, n, cin, h, w, cout, k, p, d) in SHAPES:
        if flt not in name:
            continue
        torch.manual_seed(0)
        oh, ow = h, w
        fl = 2.0 * n * oh * ow * cout * k * k * cin
        sets = []
        per = 0
        while per * len(sets) < 600e6 and len(sets) < 64:
            wp = (torch.randn(cout, cin, k, k, device=dev) * 0.05).contiguous(memory_format=torch.channels_last)
            wf, wt = ops.WCACHE.get(wp, dt)
            if op == "fwd":
                x = torch.randn(n * h * w, cin, device=dev).to(dt)
                y = torch.empty(n * oh * ow, cout, device=dev, dtype=dt)
                sets.append((lambda x=x, wf=wf, y=y: ops.conv_fwd(x, n, h, w, wf, cout, k, 1, p, d, out=y)))
                per = (x.numel() + y.numel() + wf.numel()) * 2
            else:
                dy = torch.randn(n * oh * ow, cout, device=dev).to(dt)
                dx = torch.empty(n * h * w, cin, device=dev, dtype=dt)
                sets.append((lambda dy=dy, wt=wt, dx=dx: ops.conv_dgrad(dy, n, oh, ow, wt, cin, k, 1, p, d, h, w, out=dx)))
                per = (dy.numel() + dx.numel() + wt.numel()) * 2
        line = "%-24s M=%6d N=%5d K=%6d sets=%2d |" % (name, n * oh * ow, cout if op == "fwd" else cin,
                                                      k * k * (cin if op == "fwd" else cout), len(sets))
        for c in cfgs:
            nv.load().cn_gemm_force_config(c)
            tw = gtime_sets(sets[:1], reps=20)
            tc = gtime_sets(sets)
            line += " c%d %5.1f/%5.1f us" % (c, tw * 1e6, tc * 1e6)
        nv.load().cn_gemm_force_config(-1)
        print(line + "   (warm/cold; %.1f GFLOP)" % (fl / 1e9), flush=True)
        del sets
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
