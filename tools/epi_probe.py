"""Time conv fwd / dgrad with and without the BN epilogues (and the separate BN passes they
replace) on one shape:  python tools/epi_probe.py [shape ...]"""
import sys
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
import torch
from cosnet_amd import ops
from test_gpu_kernels import _BN

dev = torch.device('cuda:0')
dt = torch.bfloat16
SH = {"l3b_1x1": (8, 256, 60, 60, 1024, 1, 1, 0, 1), "l3_1x1": (8, 1024, 60, 60, 256, 1, 1, 0, 1),
      "l3": (8, 256, 60, 60, 256, 3, 1, 2, 2), "aspp": (8, 2048, 60, 60, 512, 3, 1, 12, 12),
      "l1_1x1": (8, 256, 119, 119, 64, 1, 1, 0, 1),
      # round 3: every other conv -> BN shape of the two encoders (frame batch 2 x 4)
      "l1b_1x1": (8, 64, 119, 119, 256, 1, 1, 0, 1), "l1_3x3": (8, 64, 119, 119, 64, 3, 1, 1, 1),
      "l1_ds": (8, 64, 119, 119, 256, 1, 1, 0, 1), "l2_1x1": (8, 512, 60, 60, 128, 1, 1, 0, 1),
      "l2_3x3": (8, 128, 60, 60, 128, 3, 1, 1, 1), "l2b_1x1": (8, 128, 60, 60, 512, 1, 1, 0, 1),
      "l3_ds": (8, 512, 60, 60, 1024, 1, 1, 0, 1), "l4_1x1": (8, 2048, 60, 60, 512, 1, 1, 0, 1),
      "l4": (8, 512, 60, 60, 512, 3, 1, 4, 4), "l4b_1x1": (8, 512, 60, 60, 2048, 1, 1, 0, 1),
      "l4_ds": (8, 1024, 60, 60, 2048, 1, 1, 0, 1)}


def tm(fn, reps=30):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for name in (sys.argv[1:] or list(SH)):
    n, cin, h, w, cout, k, s, p, d = SH[name]
    x = torch.randn(n * h * w, cin, device=dev).to(dt)
    wf = (torch.randn(cout, k * k * cin, device=dev) * 0.05).to(dt)
    wt = (torch.randn(cin, k * k * cout, device=dev) * 0.05).to(dt)
    bn = _BN(cout, dev, 1)
    bni = _BN(cin, dev, 2)
    t0 = tm(lambda: ops.conv_fwd(x, n, h, w, wf, cout, k, s, p, d))
    t1 = tm(lambda: ops.conv_fwd_bn(x, n, h, w, wf, cout, k, s, p, d, bn, 2))
    c, oh, ow = ops.conv_fwd(x, n, h, w, wf, cout, k, s, p, d)
    t2 = tm(lambda: ops.bn_stats(c, bn, True, nseg=2))
    line = "%-8s fwd %7.1f  fwd_bn %7.1f  (+%5.1f)  stats pass %6.1f us" % (name, t0, t1, t1 - t0, t2)
    if s == 1:
        nh = n // 2
        dy = torch.randn(nh * oh * ow, cout, device=dev).to(dt)
        xp = x[:nh * h * w]
        st = ops.bn_stats(xp, bni, True)
        t3 = tm(lambda: ops.conv_dgrad(dy, nh, oh, ow, wt, cin, k, 1, p, d, h, w))
        t4 = tm(lambda: ops.conv_dgrad_bn(dy, nh, oh, ow, wt, cin, k, p, d, xp, st, bni))
        dz = ops.conv_dgrad(dy, nh, oh, ow, wt, cin, k, 1, p, d, h, w)
        t5 = tm(lambda: ops.bn_bwd(xp, dz, None, st, bni, act=1, want_dx=False))
        line += " | dgrad %7.1f  dgrad_bn %7.1f (+%5.1f)  reduce pass %6.1f" % (t3, t4, t4 - t3, t5)
    print(line, flush=True)
