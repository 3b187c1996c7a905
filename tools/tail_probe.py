"""Layer-3 bottleneck tail (8 frames x 60x60, conv3 256 -> 1024, BN3 + residual + ReLU): the
separate form (conv GEMM, statistics pass, apply pass) vs the two-pass GEMM form
(cn_conv_fwd_bn_relu_res), and their pieces.  Timing probe (graph replay, operand sets cycling).
usage: python tools/tail_probe.py"""
import sys

import torch

sys.path.insert(0, '.')
sys.path.insert(0, 'tools')
from cosnet_amd import ops  # noqa: E402
from gemm_cold import gtime_sets  # noqa: E402

dev = torch.device('cuda:0')
dt = torch.bfloat16
n, h, w, planes, nseg = 8, 60, 60, 256, 2
P, c4 = n * h * w, 4 * planes
bn = torch.nn.BatchNorm2d(c4).to(dev)
sets = []
for _ in range(4):
    y2 = torch.randn(P, planes, device=dev).to(dt)
    x = torch.randn(P, c4, device=dev).to(dt)
    wp = (torch.randn(c4, planes, 1, 1, device=dev) * 0.05).contiguous(memory_format=torch.channels_last)
    wf, _ = ops.WCACHE.get(wp, dt)
    mk = ops.relu_mask(P, c4, x)
    sets.append((y2, x, wf, mk))


def separate(y2, x, wf, mk):
    c, _, _ = ops.conv_fwd(y2, n, h, w, wf, c4, 1, 1, 0, 1)
    st = ops.bn_stats(c, bn, True, nseg)
    ops.bn_apply(c, st, bn, act=1, res=x, nseg=nseg, mask=mk)


def fused(y2, x, wf, mk):
    ops.conv_fwd_bn_res(y2, n, h, w, wf, c4, 1, 1, 0, 1, bn, nseg, res=x, mask=mk)


def gemm_only(y2, x, wf, mk):
    ops.conv_fwd(y2, n, h, w, wf, c4, 1, 1, 0, 1)


def gemm_stats_epi(y2, x, wf, mk):
    ops.conv_fwd_bn(y2, n, h, w, wf, c4, 1, 1, 0, 1, bn, nseg)


for name, f in (("separate: gemm+stats+apply", separate), ("fused two-pass", fused),
                ("gemm alone", gemm_only), ("gemm + stats epilogue", gemm_stats_epi)):
    t = gtime_sets([lambda s=s: f(*s) for s in sets], reps=3)
    print("%-28s %7.1f us" % (name, t * 1e6), flush=True)
