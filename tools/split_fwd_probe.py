"""The ASPP bottleneck conv forward (8 frames x 60x60, 2560 -> 256, 3x3): split over K on 256x256
tiles (cn_conv_fwd_ws) vs the unsplit 128x256 launch (cn_conv_fwd), and the conv + BN statistics
forms (split + statistics pass vs the statistics epilogue).  Timing probe (tools/gemm_cold.py's
graph-replay timer, operands cycling through > 600 MB).
usage: python tools/split_fwd_probe.py"""
import sys

import torch

sys.path.insert(0, '.')
sys.path.insert(0, 'tools')
from cosnet_amd import _native as nv  # noqa: E402
from cosnet_amd import ops  # noqa: E402
from gemm_cold import gtime_sets  # noqa: E402

dev = torch.device('cuda:0')
dt = torch.bfloat16
n, h, w, cin, cout, k = 8, 60, 60, 2560, 256, 3
M = n * h * w
bn = torch.nn.BatchNorm2d(cout).to(dev)
sets = []
while len(sets) < 4:
    x = torch.randn(M, cin, device=dev).to(dt)
    wp = (torch.randn(cout, cin, k, k, device=dev) * 0.01).contiguous(memory_format=torch.channels_last)
    wf, _ = ops.WCACHE.get(wp, dt)
    y = torch.empty(M, cout, device=dev, dtype=dt)
    ws = torch.empty(ops.fwd_split_floats(x, M, cout, k * k * cin), device=dev)
    sets.append((x, wf, y, ws))


def split(x, wf, y, ws):
    nv.call("cn_conv_fwd_ws", nv.DT_BF16, x.data_ptr(), cin, n, h, w, cin, wf.data_ptr(), cout, k, k, 1, 1,
            1, 0, y.data_ptr(), cout, h, w, ws.data_ptr(), ws.numel(), nv.stream())


def plain(x, wf, y, ws):
    nv.call("cn_conv_fwd", nv.DT_BF16, x.data_ptr(), cin, n, h, w, cin, wf.data_ptr(), cout, k, k, 1, 1, 1,
            0, y.data_ptr(), cout, h, w, nv.stream())


fl = 2.0 * M * cout * k * k * cin
for name, f in (("split-K 256x256 + reduce", split), ("unsplit 128x256", plain)):
    t = gtime_sets([lambda s=s: f(*s) for s in sets], reps=3)
    print("%-28s %7.1f us  %5.0f TF/s" % (name, t * 1e6, fl / t / 1e12), flush=True)
t = gtime_sets([lambda s=s: ops.conv_fwd_bn(s[0], n, h, w, s[1], cout, k, 1, 1, 1, bn, nseg=2) for s in sets], reps=3)
print("%-28s %7.1f us" % ("conv_fwd_bn (split + stats)", t * 1e6), flush=True)
