"""Both frames of one encoder in ONE batched pass: EncoderPairFn.

The reference calls each encoder twice per step: once on frame a (with grad) and once on
frame b under no_grad (rgbd_segmentation_RAA.py:143-148, :198-203).  Every op of the
encoder is per-sample except BatchNorm's batch statistics, so frames a and b are stacked
into one NHWC batch of 2N images: every GEMM runs with twice the rows (better MFMA tile
occupancy, half the launches) while BN statistics and running-stat updates are computed per
frame segment, a first then b, exactly as the two separate reference calls do.  The backward
(hand-written, no per-block autograd nodes) runs on the frame-a rows only, which is all the
reference differentiates.

Reference blocks: stem deeplab/residual_net.py:157-160, Bottleneck :74-96, ASPP
deeplab/deeplabv3_encoder.py:50-86.
"""
import os

import torch

from . import _native as nv
from . import ops
from .fp8 import fp8_ok
from .ops import WCACHE, as_param_grad, bn_apply, bn_bwd, bn_stats, conv_dgrad, conv_fwd, conv_wgrad

from .functions import F, _GRAD


# ---- gradient destinations ------------------------------------------------------------------
class GradSink(dict):
    """Where the hand-written encoder backward puts parameter gradients.  Plain: fresh tensors
    collected here and handed to autograd.  With a gradient arena ({param: flat fp32 slice}, the
    data-parallel bucket buffer) every gradient is written straight into its slice: the big ones
    by the producing kernels themselves (buf()), the rest copied in on assignment."""

    def __init__(self, arena=None):
        super().__init__()
        self.arena = arena

    def buf(self, p, *shape):
        if self.arena is None or p not in self.arena:
            return None
        return self.arena[p].view(*shape)

    def __setitem__(self, p, g):
        if self.arena is not None and p in self.arena:
            dst = self.arena[p]
            if g.data_ptr() != dst.data_ptr():   # not produced in place (the stem's padded dw)
                dst.as_strided(p.shape, p.stride()).copy_(g)
            return
        super().__setitem__(p, g)


# When the queued bottleneck weight gradients are issued in a single-process encoder backward:
# "end" (after the whole dgrad chain) or "layer" (after each layer's blocks: the queue's dY and
# input tensors are released per layer).  CN_WGRAD_FLUSH selects it for A/B runs.
WGRAD_FLUSH = os.environ.get("CN_WGRAD_FLUSH", "end")
# Groups of >= 2 problems with fewer than CN_WGRAD_GSPLIT tiles (128x64 units) in total run split
# over K as well (cn_conv_wgrad_grouped_ws); 0 issues the small ones one by one as split-K
# launches (A/B runs).
WGRAD_GSPLIT = int(os.environ.get("CN_WGRAD_GSPLIT", "512"))
# fp8 mode (configs[4]): the 3x3 bottleneck and ASPP weight gradients on fp8 operands
# (cn_conv_wgrad_fp8); CN_WGRAD_FP8=0 keeps them bf16 (A/B runs).
WGRAD_FP8 = os.environ.get("CN_WGRAD_FP8", "1") != "0"
# The ASPP's three atrous convs in one grouped launch (cn_conv_fwd_bn_grouped, train mode, bf16 /
# fp32): measured level with the three launches in the two-stream step (the depth stream already
# fills the CUs a one-round launch leaves idle; profiles/r06_aspp_grouped_fp8_stats_ab.txt), so
# off by default; CN_ASPP_GROUPED=1 selects it.
ASPP_GROUPED = os.environ.get("CN_ASPP_GROUPED", "0") == "1"
# fp8 mode: the BN statistics of the long-K narrow fp8 convs (fuse_stats) from the fp8 GEMM's
# epilogue (cn_conv_fwd_fp8_bn) instead of their own pass: measured 0.8 % SLOWER on the configs[4]
# step (the fp8 tiles' epilogue is long next to their K loop), so off by default;
# CN_FP8_FUSE_STATS=1 selects it.
FP8_FUSE_STATS = os.environ.get("CN_FP8_FUSE_STATS", "0") == "1"
# TIMING PROBE ONLY (results are wrong): CN_PROBE_SKIP_APPLY=1 / 2 / 3 drops the bn1 / bn2 / both
# BN + ReLU apply passes of every bottleneck (the next conv reads the raw conv output) -- the
# upper bound of what folding those applies into the consumer conv's operand path could save
# (VERDICT r4 "next" #4; profiles/r05_bn_fold_bound.txt).
_PROBE_SKIP = int(os.environ.get("CN_PROBE_SKIP_APPLY", "0"))


# The per-module path (functions.StemFn / BottleneckFn / ASPPFn: frames of different sizes, e.g.
# configs[3]'s 1 target vs 5 references) runs the block functions below with one segment and
# without fp8 (its calls bracket no Fp8Acts pass): _FP8_OFF[0] is set around them.
_FP8_OFF = [False]


def fp8_of(mod):
    """The fp8 context a module's convs use (None: bf16 / fp32 operands)."""
    return None if _FP8_OFF[0] else getattr(mod, "_cn_fp8", None)


class no_fp8:
    def __enter__(self):
        self.prev = _FP8_OFF[0]
        _FP8_OFF[0] = True

    def __exit__(self, *a):
        _FP8_OFF[0] = self.prev
        return False


def _layer_index(enc):
    """id(block) -> index of its ResNet layer."""
    bb = enc.backbone
    return {id(blk): i for i, layer in enumerate((bb.layer1, bb.layer2, bb.layer3, bb.layer4))
            for blk in layer}


class WgradQueue:
    """Weight gradients of the bottlenecks, run after the dgrad chain of an encoder backward (or of
    one data-parallel segment) as grouped launches: the same conv of consecutive bottlenecks has
    one shape, so G of them form one launch of G x tiles workgroups that each run the whole K --
    no split-K slabs and no reduce launch -- instead of G split-K launches + G reduces on the
    critical chain (the bottleneck weight gradients cost 5.1 ms of the 32.9 ms step issued one
    by one, profiles/r03_skip_wgrad_probe.txt).  They are issued after the chain on the same
    stream (on a side stream they slowed the chain, profiles/r03_wgrad_side_stream_ab.txt);
    their inputs (dY of the conv, its saved input) stay referenced here until flush()."""

    def __init__(self):
        self.jobs = {}

    def add(self, x, n, h, w, cin, dy, oh, ow, cout, k, stride, pad, dil, dw=None, f8=None):
        """f8 = (x8, x_state, dy8, dy_state): run this weight gradient on fp8 operands (configs[4],
        grouped with the other fp8 jobs of its shape; cn_conv_wgrad_fp8)."""
        if dw is None:
            dw = torch.empty((cout, k * k * cin), dtype=torch.float32, device=x.device)
        if f8 is not None:
            x8, xs, dy8, ds = f8
            key = ("f8", n, h, w, cin, ops.ld(x8), oh, ow, cout, ops.ld(dy8), k, stride, pad, dil)
            self.jobs.setdefault(key, []).append((x8, xs, dy8, ds, dw))
            return dw
        key = (x.dtype, n, h, w, cin, ops.ld(x), oh, ow, cout, ops.ld(dy), k, stride, pad, dil)
        self.jobs.setdefault(key, []).append((x, dy, dw))
        return dw

    def flush(self):
        for key, jobs in self.jobs.items():
            _, n, h, w, cin, _, oh, ow, cout, _, k, stride, pad, dil = key
            if key[0] == "f8":
                for i in range(0, len(jobs), ops.GROUP_MAX):
                    ops.conv_wgrad_fp8(jobs[i:i + ops.GROUP_MAX], n, h, w, cin, oh, ow, cout, k,
                                       stride, pad, dil)
                continue
            # grouped when >= 3 problems give >= 128 workgroups of 128x64 (two layer-4 1x1
            # weight gradients: 2 x 55 us split-K vs 137 us grouped; three: 160 vs 144 us,
            # profiles/r03_wgrad_l4_1x1.txt)
            tiles = -(-cout // 128) * -(-(k * k * cin) // 64)
            for i in range(0, len(jobs), ops.GROUP_MAX):
                chunk = jobs[i:i + ops.GROUP_MAX]
                if len(chunk) >= 2 and tiles * len(chunk) < WGRAD_GSPLIT:
                    # small shapes (layers 1-2): the group split over K as well -- one GEMM and
                    # one reduce launch instead of a split-K GEMM + reduce per problem
                    ops.conv_wgrad_grouped(chunk, n, h, w, cin, oh, ow, cout, k, stride, pad, dil,
                                           split=True)
                elif len(chunk) >= 3 and tiles * len(chunk) >= 128:
                    ops.conv_wgrad_grouped(chunk, n, h, w, cin, oh, ow, cout, k, stride, pad, dil)
                else:
                    for x, dy, dw in chunk:
                        conv_wgrad(x, n, h, w, cin, dy, oh, ow, cout, k, stride, pad, dil, dw=dw)
        self.jobs = {}


# ---- segment helpers -----------------------------------------------------------------------
class SegStats:
    """BN statistics of nseg stacked frame segments: mean / invstd [nseg*C]; [i] -> segment i."""

    def __init__(self, stats, nseg, c):
        self.mean, self.invstd = stats
        self.nseg, self.c = nseg, c

    def __len__(self):
        return self.nseg

    def __getitem__(self, i):
        return ops.seg_of((self.mean, self.invstd), i, self.c)


def seg_stats(x, bn, training, nseg):
    """Per-segment (frame) BN statistics in one launch pair; running stats updated segment by
    segment."""
    return SegStats(bn_stats(x, bn, training, nseg=nseg), nseg, x.shape[1])


def fuse_stats(cout, kdim):
    """The BN-statistics epilogue pays off on long-K, narrow convs (measured per shape,
    tools/epi_probe.py: layer-3 1x1 1024->256 34 vs 40 us, 3x3 52 vs 56 us, ASPP 446 vs 480 us);
    on short-K / wide outputs (256->1024 1x1: 61 vs 51 us) the separate pass is cheaper."""
    return kdim >= 1024 and cout <= 512


def fuse_bwd(cin, kdim):
    """Same for the dgrad epilogue that reduces the BN backward (43 vs 45 us on the layer-3 3x3,
    30 vs 34 us on the 256->1024 1x1; a loss on 1024-wide outputs)."""
    return kdim >= 1024 and cin <= 256


def conv_bn(x, n, h, w, wf, cout, k, stride, pad, dil, bn, training, nseg, bias=None, weight=None,
            q8=None):
    """conv -> raw output c and the BN statistics of c per segment.  Train mode: the statistics
    come out of the conv's GEMM epilogue where that is cheaper (ops.conv_fwd_bn, no pass over c),
    else a separate statistics pass; eval: running statistics.  fp8 mode (configs[4]): the
    conv GEMM takes e4m3 operands (cosnet_amd/fp8.py), statistics from its epilogue by the same
    rule (ops.conv_fwd_fp8_bn) or the separate pass; with a list q8 the e4m3 input copy is
    appended to it as Fp8Acts.saved() (for the fp8 weight gradient)."""
    cin = wf.shape[1] // (k * k)
    ctx = fp8_of(bn)
    if weight is not None and ctx is not None and fp8_ok(x, cin) and x.shape[0] > 64:
        x8, xs = ctx.acts.quant(x, id(weight))
        if q8 is not None:
            q8.append(ctx.acts.saved(x8, xs))
        wf8, ws = ctx.weights.get(weight)
        if training and FP8_FUSE_STATS and fuse_stats(cout, wf.shape[1]):
            # the statistics from the fp8 GEMM's epilogue, as the bf16 path takes them (round 6)
            c, oh, ow, st = ops.conv_fwd_fp8_bn(x8, n, h, w, wf8, cout, k, stride, pad, dil, xs, ws,
                                                bn, nseg, bias=bias)
            return c, oh, ow, SegStats(st, nseg, cout)
        c, oh, ow = ops.conv_fwd_fp8(x8, n, h, w, wf8, cout, k, stride, pad, dil, xs, ws, bias=bias)
        return c, oh, ow, seg_stats(c, bn, training, nseg)
    if training and fuse_stats(cout, wf.shape[1]):
        c, oh, ow, st = ops.conv_fwd_bn(x, n, h, w, wf, cout, k, stride, pad, dil, bn, nseg, bias=bias)
        return c, oh, ow, SegStats(st, nseg, cout)
    c, oh, ow = conv_fwd(x, n, h, w, wf, cout, k, stride, pad, dil, bias=bias)
    return c, oh, ow, seg_stats(c, bn, training, nseg)


def seg_apply(x, stats, bn, act=0, prelu=None, res=None, xr=None, rstats=None, rbn=None, out=None,
              fp8_key=None, mask=None):
    """BN apply; in fp8 mode with fp8_key (the output feeds fp8 convs) also the e4m3 copy of the
    output in the same pass (delayed scaling; a first use calibrates by a separate pass); with
    mask (ops.relu_mask) also the ReLU mask bits the backward reads instead of the output."""
    rs = None if rstats is None else (rstats.mean, rstats.invstd)
    ctx = fp8_of(bn)
    if fp8_key is None or ctx is None or x.dtype != torch.bfloat16:
        return bn_apply(x, (stats.mean, stats.invstd), bn, act=act, prelu=prelu, res=res, xr=xr,
                        rstats=rs, rbn=rbn, out=out, nseg=stats.nseg, mask=mask)
    st = ctx.acts.ready(fp8_key, x.device)
    if st is None:
        y = bn_apply(x, (stats.mean, stats.invstd), bn, act=act, prelu=prelu, res=res, xr=xr,
                     rstats=rs, rbn=rbn, out=out, nseg=stats.nseg, mask=mask)
        ctx.acts.quant(y, fp8_key)
        return y
    y8 = torch.empty(tuple(x.shape), dtype=torch.uint8, device=x.device)
    y = bn_apply(x, (stats.mean, stats.invstd), bn, act=act, prelu=prelu, res=res, xr=xr, rstats=rs,
                 rbn=rbn, out=out, nseg=stats.nseg, out8=y8, qstate=st, mask=mask)
    ctx.acts.register(y, y8, st)
    return y


# ---- stem --------------------------------------------------------------------------------------
def stem_fwd(res, imgs, nseg, dt, rec):
    n1, cimg, h, w = imgs[0].shape
    n = n1 * len(imgs)
    x = torch.empty((n * h * w, 8), dtype=dt, device=imgs[0].device)
    for i, img in enumerate(imgs):
        nv.call("cn_nchw_to_nhwc", nv.dtype_code(dt), img.data_ptr(), n1, cimg, h, w, 8,
                x[i * n1 * h * w:].data_ptr(), nv.stream())
    wf, _ = WCACHE.get(res.conv1.weight, dt, cin_pad=8, need_t=False)
    c, oh, ow, st = conv_bn(x, n, h, w, wf, 64, 7, 2, 3, 1, res.bn1, res.training, nseg)
    y = seg_apply(c, st, res.bn1, act=1)
    ph, pw = ops.pool_out(oh), ops.pool_out(ow)
    out = torch.empty((n * ph * pw, 64), dtype=dt, device=x.device)
    am = torch.empty((n * ph * pw * 64,), dtype=torch.uint8, device=x.device)
    nv.call("cn_maxpool_fwd", nv.dtype_code(dt), y.data_ptr(), n, oh, ow, 64, ph, pw, 3, 2, 1,
            out.data_ptr(), am.data_ptr(), nv.stream())
    if rec is not None:
        rec.append(("stem", res, (x, c, y, am, st), (n1, cimg, h, w, oh, ow, ph, pw)))
    return out, (n, ph, pw)


def stem_bwd(item, dout, grads):
    _, res, (x, c, y, am, st), (n1, cimg, h, w, oh, ow, ph, pw) = item
    pa = n1 * oh * ow
    dy = torch.empty((pa, 64), dtype=dout.dtype, device=dout.device)
    nv.call("cn_maxpool_bwd", ops.dtc(dout), dout.data_ptr(), am.data_ptr(), n1, oh, ow, 64, ph,
            pw, 3, 2, 1, dy.data_ptr(), nv.stream())
    dc, dg, db, _ = bn_bwd(c[:pa], dy, None, st[0], res.bn1, act=1,
                           dgamma=grads.buf(res.bn1.weight, 64), dbeta=grads.buf(res.bn1.bias, 64))
    dw = conv_wgrad(x[:n1 * h * w], n1, h, w, 8, dc, oh, ow, 64, 7, 2, 3, 1)
    grads[res.conv1.weight] = dw.view(64, 7, 7, 8)[..., :cimg].permute(0, 3, 1, 2)
    grads[res.bn1.weight] = dg
    grads[res.bn1.bias] = db


def fp8_dgrad_ok(dy, k):
    """fp8 dgrad (e5m2 dY x e4m3 W^T) for the compute-heavy stride-1 convs: K = k*k*Cout >= 2304
    (the layer-3/4 3x3 convs, the ASPP convs); the short-K 1x1 dgrads are HBM-bound and gain
    nothing from a 2x MFMA rate."""
    return (dy.dtype == torch.bfloat16 and k * k * dy.shape[1] >= 2304 and dy.shape[1] % 16 == 0
            and ops.ld(dy) % 16 == 0 and dy.shape[0] > 64)


def wgrad_f8(ctx, q8, dy, rows, k, weight, cin):
    """fp8 operands for a weight gradient (configs[4]) when both exist: the forward's e4m3 input
    copy (q8 = Fp8Acts.saved(), frame-a `rows`) and an e5m2 output gradient the fp8 dgrad quantises
    (fp8_dgrad_ok; the same pass-cached copy serves both).  (x8, x_state, dy8, dy_state) or None."""
    if ctx is None or not q8 or not fp8_dgrad_ok(dy, k) or cin % 16:
        return None
    x8, handle, slot = q8[0]
    dy8, ds = ctx.grads.quant(dy, ("dgrad", id(weight)))
    return x8[:rows], handle.state(slot), dy8, ds


def wgrad_now(x, n, h, w, cin, dy, oh, ow, cout, k, stride, pad, dil, dw=None, f8=None):
    """One weight gradient issued now: fp8 (f8 from wgrad_f8) or the bf16 / fp32 path."""
    if f8 is None:
        return conv_wgrad(x, n, h, w, cin, dy, oh, ow, cout, k, stride, pad, dil, dw=dw)
    if dw is None:
        dw = torch.empty((cout, k * k * cin), dtype=torch.float32, device=dy.device)
    x8, xs, dy8, ds = f8
    ops.conv_wgrad_fp8([(x8, xs, dy8, ds, dw)], n, h, w, cin, oh, ow, cout, k, stride, pad, dil)
    return dw


def dgrad(dy, n, oh, ow, wt, cin, k, pad, dil, h, w, weight, ctx, out=None, accumulate=False):
    """Stride-1 conv dgrad: in fp8 mode (ctx, BASELINE configs[4]) e5m2 output gradients
    (delayed scaling, ctx.grads) x the e4m3 transposed weight on the block-scaled MFMA."""
    if ctx is not None and fp8_dgrad_ok(dy, k):
        dy8, ds = ctx.grads.quant(dy, ("dgrad", id(weight)))
        wt8, ws = ctx.weights.get_t(weight, wt)
        return ops.conv_dgrad_fp8(dy8, n, oh, ow, wt8, cin, k, pad, dil, h, w, ds, ws, out=out,
                                  accumulate=accumulate)
    return conv_dgrad(dy, n, oh, ow, wt, cin, k, 1, pad, dil, h, w, out=out, accumulate=accumulate)


def dgrad_bn_bwd(dy, n, oh, ow, wt, cin, k, pad, dil, x, stats, bn, grads, weight=None, ctx=None):
    """Stride-1 conv dgrad followed by the backward of the BN + ReLU (mask from x) that fed the
    conv: returns (dx of the BN input, dgamma, dbeta)."""
    dgo, dbo = grads.buf(bn.weight, cin), grads.buf(bn.bias, cin)
    if ctx is not None and fp8_dgrad_ok(dy, k):
        dyb = dgrad(dy, n, oh, ow, wt, cin, k, pad, dil, oh, ow, weight, ctx)
        dx, dg, db, _ = bn_bwd(x, dyb, None, stats, bn, act=1, dgamma=dgo, dbeta=dbo)
        return dx, dg, db
    if fuse_bwd(cin, wt.shape[1]):
        dyb, dg, db = ops.conv_dgrad_bn(dy, n, oh, ow, wt, cin, k, pad, dil, x, stats, bn,
                                        dgamma=dgo, dbeta=dbo)
        return ops.bn_bwd_apply(x, dyb, stats, bn, dg, db), dg, db
    dyb = conv_dgrad(dy, n, oh, ow, wt, cin, k, 1, pad, dil, oh, ow)
    dx, dg, db, _ = bn_bwd(x, dyb, None, stats, bn, act=1, dgamma=dgo, dbeta=dbo)
    return dx, dg, db


# ---- bottleneck ----------------------------------------------------------------------------------
def bottleneck_fwd(blk, x, geo, nseg, rec):
    n, h, w = geo
    dt = x.dtype
    tr = blk.training
    s, d = blk.stride, blk.dilation
    planes = blk.conv1.weight.shape[0]
    w1f, w1t = WCACHE.get(blk.conv1.weight, dt)
    w2f, w2t = WCACHE.get(blk.conv2.weight, dt)
    w3f, w3t = WCACHE.get(blk.conv3.weight, dt)
    c1, oh, ow, st1 = conv_bn(x, n, h, w, w1f, planes, 1, s, 0, 1, blk.bn1, tr, nseg,
                              weight=blk.conv1.weight)
    y1 = c1 if _PROBE_SKIP & 1 else seg_apply(c1, st1, blk.bn1, act=1, fp8_key=id(blk.conv2.weight))
    # the e4m3 input copy is kept for the backward only when the fp8 weight gradient reads it
    q2 = [] if rec is not None and WGRAD_FP8 else None
    c2, _, _, st2 = conv_bn(y1, n, oh, ow, w2f, planes, 3, 1, d, d, blk.bn2, tr, nseg,
                            weight=blk.conv2.weight, q8=q2)
    y2 = c2 if _PROBE_SKIP & 2 else seg_apply(c2, st2, blk.bn2, act=1, fp8_key=id(blk.conv3.weight))
    c3, _, _, st3 = conv_bn(y2, n, oh, ow, w3f, 4 * planes, 1, 1, 0, 1, blk.bn3, tr, nseg,
                            weight=blk.conv3.weight)
    cd = std = wdt = None
    # the backward of the residual BN + ReLU needs only y > 0: kept as bits (1/16 of y's bytes),
    # read by bn_bwd(act=4) instead of y (deeplab/residual_net.py:107-109)
    mk = ops.relu_mask(c3.shape[0], 4 * planes, c3) if rec is not None else None
    if blk.downsample is not None:
        wdf, wdt = WCACHE.get(blk.downsample[0].weight, dt)
        bnd = blk.downsample[1]
        cd, _, _, std = conv_bn(x, n, h, w, wdf, 4 * planes, 1, s, 0, 1, bnd, tr, nseg,
                                weight=blk.downsample[0].weight)
        y = seg_apply(c3, st3, blk.bn3, act=1, xr=cd, rstats=std, rbn=bnd, fp8_key=("out", id(blk)),
                      mask=mk)
    else:
        y = seg_apply(c3, st3, blk.bn3, act=1, res=x, fp8_key=("out", id(blk)), mask=mk)
    if rec is not None:
        rec.append(("block", blk, (x, c1, y1, c2, y2, c3, cd, mk, st1, st2, st3, std, w1t, w2t, w3t, wdt, q2),
                    (n // nseg, h, w, oh, ow, s, d, planes, x.shape[1])))
    return y, (n, oh, ow)


def bottleneck_bwd(item, dy, grads, need_dx=True, wq=None):
    """Backward of one bottleneck; with a WgradQueue the four weight gradients are queued (their
    dW buffers are registered in `grads` now and filled by wq.flush())."""
    _, blk, sv, (n, h, w, oh, ow, s, d, planes, cin) = item
    wgrad = conv_wgrad if wq is None else wq.add
    x, c1, y1, c2, y2, c3, cd, mk, st1, st2, st3, std, w1t, w2t, w3t, wdt, q2 = sv
    pi, po = n * h * w, n * oh * ow                     # frame-a rows in / out
    x, c1, y1, c2, y2, c3, mk = x[:pi], c1[:po], y1[:po], c2[:po], y2[:po], c3[:po], mk[:po]
    has_down = cd is not None
    dx = None
    g3o, b3o = grads.buf(blk.bn3.weight, 4 * planes), grads.buf(blk.bn3.bias, 4 * planes)
    if has_down:
        cd = cd[:po]
        dc3, dg3, db3, _ = bn_bwd(c3, dy, mk, st3[0], blk.bn3, act=4, dgamma=g3o, dbeta=b3o)
        dcd, _, _, _ = bn_bwd(cd, dy, mk, std[0], blk.downsample[1], act=4)
    else:
        dx = torch.empty_like(x)
        dc3, dg3, db3, _ = bn_bwd(c3, dy, mk, st3[0], blk.bn3, act=4, dres=dx, dgamma=g3o, dbeta=b3o)
    dw3 = wgrad(y2, n, oh, ow, planes, dc3, oh, ow, 4 * planes, 1, 1, 0, 1,
                dw=grads.buf(blk.conv3.weight, 4 * planes, planes))
    # dgrads, fused with the reduction of the backward of the BN + ReLU that fed the conv where
    # that is cheaper (fuse_bwd)
    f8 = fp8_of(blk.bn2)
    dc2, dg2, db2 = dgrad_bn_bwd(dc3, n, oh, ow, w3t, planes, 1, 0, 1, c2, st2[0], blk.bn2, grads,
                                 weight=blk.conv3.weight, ctx=f8)
    # configs[4]: e5m2 dc2 (shared with conv2's fp8 dgrad below) x the forward's e4m3 y1
    w8 = wgrad_f8(f8, q2, dc2, po, 3, blk.conv2.weight, planes) if WGRAD_FP8 else None
    dw2 = (wgrad if wq is not None else wgrad_now)(
        y1, n, oh, ow, planes, dc2, oh, ow, planes, 3, 1, d, d,
        dw=grads.buf(blk.conv2.weight, planes, 9 * planes), f8=w8)
    dc1, dg1, db1 = dgrad_bn_bwd(dc2, n, oh, ow, w2t, planes, 3, d, d, c1, st1[0], blk.bn1, grads,
                                 weight=blk.conv2.weight, ctx=f8)
    dw1 = wgrad(x, n, h, w, cin, dc1, oh, ow, planes, 1, s, 0, 1,
                dw=grads.buf(blk.conv1.weight, planes, cin))
    if need_dx:
        dx = conv_dgrad(dc1, n, oh, ow, w1t, cin, 1, s, 0, 1, h, w, out=dx, accumulate=dx is not None)
    if has_down:
        dwd = wgrad(x, n, h, w, cin, dcd, oh, ow, 4 * planes, 1, s, 0, 1,
                    dw=grads.buf(blk.downsample[0].weight, 4 * planes, cin))
        grads[blk.downsample[0].weight] = as_param_grad(dwd, blk.downsample[0].weight)
        if need_dx:
            conv_dgrad(dcd, n, oh, ow, wdt, cin, 1, s, 0, 1, h, w, out=dx, accumulate=True)
    grads[blk.conv1.weight] = as_param_grad(dw1, blk.conv1.weight)
    grads[blk.conv2.weight] = as_param_grad(dw2, blk.conv2.weight)
    grads[blk.conv3.weight] = as_param_grad(dw3, blk.conv3.weight)
    grads[blk.bn1.weight], grads[blk.bn1.bias] = dg1, db1
    grads[blk.bn2.weight], grads[blk.bn2.bias] = dg2, db2
    grads[blk.bn3.weight], grads[blk.bn3.bias] = dg3, db3
    return dx


# ---- ASPP ------------------------------------------------------------------------------------------
def aspp_fwd(mod, x, geo, nseg, rec):
    n, h, w = geo
    hw = h * w
    P = n * hw
    dt = x.dtype
    tr = mod.training
    dev = x.device
    cat = torch.empty((P, 2560), dtype=dt, device=dev)
    pool = torch.empty((n, 2048), dtype=dt, device=dev)
    ops.avgpool(x, n, hw, 1.0 / hw, pool)
    wcf, wct = WCACHE.get(mod.conv.weight, dt)
    cp, _, _, stp = conv_bn(pool, n, 1, 1, wcf, 512, 1, 1, 0, 1, mod.bn_x, tr, nseg, bias=mod.conv.bias)
    yp = seg_apply(cp, stp, mod.bn_x, act=1)
    nv.call("cn_bcast_rows", ops.dtc(yp), yp.data_ptr(), n, hw, 512, 1.0, cat.data_ptr(), 2560, 0,
            nv.stream())
    # fp8 mode: the concat's e4m3 copy for the bottleneck conv, written by the branches' applies
    # (one delayed-scaling state for the whole concat; the pooled slice by a quantise pass)
    cat8 = qst = None
    ctx = fp8_of(mod) if dt == torch.bfloat16 else None
    if ctx is not None:
        qst = ctx.acts.ready(("cat", id(mod)), dev)
        if qst is not None:
            cat8 = torch.empty((P, 2560), dtype=torch.uint8, device=dev)
            ops.fp8_quant(cat[:, :512], qst, ops.FP8_DELAYED, out=cat8[:, :512])
    convs = [(mod.conv2d_0, mod.bn_0, 1, 0)] + [
        (getattr(mod, "conv2d_%d" % (i + 1)), getattr(mod, "bn_%d" % (i + 1)), 3, dd)
        for i, dd in enumerate(mod.cn_dilations)]
    # the atrous branches as one grouped launch (train mode, statistics from the epilogue, not
    # fp8): each branch's launch alone is one round of the chip set by its tiles that skip no tap
    grouped = {}
    if (tr and ctx is None and ASPP_GROUPED and fuse_stats(512, 9 * x.shape[1])
            and all(dd > 0 for (_, _, _, dd) in convs[1:])):
        at = convs[1:]
        outs = ops.conv_fwd_bn_grouped(x, n, h, w, [WCACHE.get(cm.weight, dt)[0] for (cm, _, _, _) in at],
                                       512, 3, [dd for (_, _, _, dd) in at], [bnm for (_, bnm, _, _) in at],
                                       nseg, biases=[cm.bias for (cm, _, _, _) in at])
        for bi, (y_, st_) in enumerate(outs):
            grouped[bi + 1] = (y_, SegStats(st_, nseg, 512))
    cs, sts, wts, q8s = [], [], [], []
    for bi, (cm, bnm, k, dd) in enumerate(convs):
        wf, wt = WCACHE.get(cm.weight, dt)
        q = [] if rec is not None and WGRAD_FP8 else None
        if bi in grouped:
            ci, st = grouped[bi]
        else:
            ci, _, _, st = conv_bn(x, n, h, w, wf, 512, k, 1, dd, max(dd, 1), bnm, tr, nseg, bias=cm.bias,
                                   weight=cm.weight, q8=q)
        q8s.append(q)
        sl = slice(512 * (bi + 1), 512 * (bi + 2))
        if cat8 is not None:
            bn_apply(ci, (st.mean, st.invstd), bnm, act=1, out=cat[:, sl], nseg=st.nseg,
                     out8=cat8[:, sl], qstate=qst)
        else:
            seg_apply(ci, st, bnm, act=1, out=cat[:, sl])
        cs.append(ci)
        sts.append(st)
        wts.append(wt)
    if cat8 is not None:
        ctx.acts.register(cat, cat8, qst)
    elif ctx is not None:
        ctx.acts.quant(cat, ("cat", id(mod)))   # first use: calibrates the concat's scale
    wbf, wbt = WCACHE.get(mod.bottleneck.weight, dt)
    qb = [] if rec is not None and WGRAD_FP8 else None
    cb, _, _, stb = conv_bn(cat, n, h, w, wbf, 256, 3, 1, 1, 1, mod.bn, tr, nseg, bias=mod.bottleneck.bias,
                            weight=mod.bottleneck.weight, q8=qb)
    out = seg_apply(cb, stb, mod.bn, act=2, prelu=mod.prelu.weight)
    if rec is not None:
        rec.append(("aspp", mod, (x, pool, cp, yp, stp, wct, cs, sts, wts, cat, cb, stb, wbt, out, q8s, qb),
                    (n // nseg, h, w, [(k, dd) for (_, _, k, dd) in convs])))
    return out


def aspp_bwd(item, dout, grads):
    _, mod, sv, (n, h, w, kd) = item
    x, pool, cp, yp, stp, wct, cs, sts, wts, cat, cb, stb, wbt, out, q8s, qb = sv
    hw = h * w
    P = n * hw
    f8 = fp8_of(mod.bn)
    use8 = f8 is not None and WGRAD_FP8
    x, cat, cb, out = x[:P], cat[:P], cb[:P], out[:P]
    pool, cp, yp = pool[:n], cp[:n], yp[:n]
    pw = mod.prelu.weight
    dcb, dgb, dbb, dpr = bn_bwd(cb, dout, out, stb[0], mod.bn, act=2, prelu=pw,
                                dgamma=grads.buf(mod.bn.weight, 256), dbeta=grads.buf(mod.bn.bias, 256),
                                dprelu=grads.buf(pw, 1))
    grads[mod.bottleneck.weight] = as_param_grad(
        wgrad_now(cat, n, h, w, 2560, dcb, h, w, 256, 3, 1, 1, 1,
                  dw=grads.buf(mod.bottleneck.weight, 256, 9 * 2560),
                  f8=wgrad_f8(f8, qb, dcb, P, 3, mod.bottleneck.weight, 2560) if use8 else None),
        mod.bottleneck.weight)
    grads[mod.bottleneck.bias] = ops.colsum(dcb, out=grads.buf(mod.bottleneck.bias, 256))
    grads[mod.bn.weight], grads[mod.bn.bias], grads[pw] = dgb, dbb, dpr
    dcat = dgrad(dcb, n, h, w, wbt, 2560, 3, 1, 1, h, w, mod.bottleneck.weight, f8)
    dx = None
    bns = [mod.bn_0, mod.bn_1, mod.bn_2, mod.bn_3]
    cms = [mod.conv2d_0, mod.conv2d_1, mod.conv2d_2, mod.conv2d_3]
    for bi, ((k, dd), ci, st, wt) in enumerate(zip(kd, cs, sts, wts)):
        sl = slice(512 * (bi + 1), 512 * (bi + 2))
        dci, dgi, dbi, _ = bn_bwd(ci[:P], dcat[:, sl], None, st[0], bns[bi], act=1,
                                  dgamma=grads.buf(bns[bi].weight, 512), dbeta=grads.buf(bns[bi].bias, 512))
        grads[cms[bi].weight] = as_param_grad(
            wgrad_now(x, n, h, w, 2048, dci, h, w, 512, k, 1, dd, max(dd, 1),
                      dw=grads.buf(cms[bi].weight, 512, k * k * 2048),
                      f8=wgrad_f8(f8, q8s[bi], dci, P, k, cms[bi].weight, 2048) if use8 else None),
            cms[bi].weight)
        grads[cms[bi].bias] = ops.colsum(dci, out=grads.buf(cms[bi].bias, 512))
        grads[bns[bi].weight], grads[bns[bi].bias] = dgi, dbi
        dx = dgrad(dci, n, h, w, wt, 2048, k, dd, max(dd, 1), h, w, cms[bi].weight, f8, out=dx,
                   accumulate=dx is not None)
    dyp = torch.empty((n, 512), dtype=dout.dtype, device=dout.device)
    ops.avgpool(dcat[:, :512], n, hw, 1.0, dyp)
    dcp, dgx, dbx, _ = bn_bwd(cp, dyp, None, stp[0], mod.bn_x, act=1,
                              dgamma=grads.buf(mod.bn_x.weight, 512), dbeta=grads.buf(mod.bn_x.bias, 512))
    grads[mod.conv.weight] = as_param_grad(conv_wgrad(pool, n, 1, 1, 2048, dcp, 1, 1, 512, 1, 1, 0, 1,
                                                      dw=grads.buf(mod.conv.weight, 512, 2048)),
                                           mod.conv.weight)
    grads[mod.conv.bias] = ops.colsum(dcp, out=grads.buf(mod.conv.bias, 512))
    grads[mod.bn_x.weight], grads[mod.bn_x.bias] = dgx, dbx
    dpool = conv_dgrad(dcp, n, 1, 1, wct, 2048, 1, 1, 0, 1, 1, 1)
    nv.call("cn_bcast_rows", ops.dtc(dpool), dpool.data_ptr(), n, hw, 2048, 1.0 / hw,
            dx.data_ptr(), ops.ld(dx), 1, nv.stream())
    return dx


# ---- the Function -----------------------------------------------------------------------------
class EncoderPairFn(F):
    """EncoderPairFn.apply(img_a, img_b, enc, *enc_params) -> (feats_a, feats_b),
    [N*h*w, 256] NHWC each; feats_b carries no gradient (the reference's no_grad call)."""

    @staticmethod
    def forward(ctx, img_a, img_b, enc, *params):
        dt = getattr(enc, "_cn_dtype", torch.bfloat16)
        fp8 = getattr(enc, "_cn_fp8", None)
        rec = [] if (_GRAD[0] and any(ctx.needs_input_grad[3:])) else None
        nseg = 2
        if fp8 is not None:
            fp8.acts.begin()
        x, geo = stem_fwd(enc.backbone, (img_a, img_b), nseg, dt, rec)
        for layer in (enc.backbone.layer1, enc.backbone.layer2, enc.backbone.layer3, enc.backbone.layer4):
            for blk in layer:
                x, geo = bottleneck_fwd(blk, x, geo, nseg, rec)
        out = aspp_fwd(enc.aspp, x, geo, nseg, rec)
        if fp8 is not None:
            fp8.acts.end()
        half = out.shape[0] // 2
        ctx.rec = rec
        ctx.params = params
        ctx.enc = enc
        ctx.training = enc.training
        ctx.defer = getattr(enc, "_cn_defer", None) if rec is not None else None
        ctx.set_materialize_grads(False)
        fa, fb = out[:half], out[half:]
        ctx.mark_non_differentiable(fb)
        return fa, fb

    @staticmethod
    def backward(ctx, dfa, dfb):
        rec = ctx.rec
        if rec is None or dfa is None:
            return (None,) * (3 + len(ctx.params))
        if not ctx.training:
            raise RuntimeError("backward through BatchNorm is implemented for train mode only")
        dfa = dfa if dfa.stride(1) == 1 else dfa.contiguous()
        ctx.rec = None
        if ctx.defer is not None:
            # data-parallel step: the encoder backward runs later, segment by segment, each
            # segment's gradients all-reduced while the next one computes (DeferredEncoderBwd)
            ctx.defer.stash(rec, dfa)
            return (None,) * (3 + len(ctx.params))
        grads = GradSink()
        f8 = getattr(ctx.enc, "_cn_fp8", None)
        if f8 is not None:
            f8.grads.begin()
        wq = WgradQueue()
        dx = aspp_bwd(rec.pop(), dfa, grads)
        stem = rec[0]
        blocks = rec[1:]
        del rec[:]                         # each block's saved tensors die with its backward
        layer_of = _layer_index(ctx.enc)
        while blocks:
            item = blocks.pop()
            dx = bottleneck_bwd(item, dx, grads, wq=wq)
            # WGRAD_FLUSH "layer": issue the queued weight gradients after the last (first in
            # backward order) block of each layer, releasing their dY / input tensors there
            if WGRAD_FLUSH == "layer" and (not blocks or layer_of[id(blocks[-1][1])] != layer_of[id(item[1])]):
                wq.flush()
            del item
        stem_bwd(stem, dx, grads)
        wq.flush()
        if f8 is not None:
            f8.grads.end()   # advance the gradient scales from this backward's amax
        return (None, None, None) + tuple(grads.get(p) for p in ctx.params)


class DeferredEncoderBwd:
    """The encoder backward of a data-parallel step, split into segments that write their
    gradients straight into the gradient arena (one bucket each).  The autograd pass only stashes
    the incoming feature gradient and the saved activations (EncoderPairFn.backward); TrainStep
    then runs run(0), run(1), ... and all-reduces bucket k while segment k+1 computes.

    Segments (reverse layer order): [ASPP + layer4], layer3 (in halves when it is deep), then
    [layer2 + layer1 + stem]."""

    def __init__(self, enc, arena):
        self.enc = enc
        self.arena = arena
        self.rec = self.dfa = self.dx = None
        bb = enc.backbone
        l3 = list(bb.layer3)
        l3_rev = list(reversed(l3))
        if len(l3) > 10:
            h = len(l3) // 2
            mid = [l3_rev[:h], l3_rev[h:]]
        else:
            mid = [l3_rev]
        # each segment: list of ("aspp" | block | "stem") in backward order
        self.plan = ([["aspp"] + list(reversed(list(bb.layer4)))] + mid +
                     [list(reversed(list(bb.layer2))) + list(reversed(list(bb.layer1))) + ["stem"]])

    def segment_params(self, k):
        """Parameters whose gradients segment k produces (its bucket), in production order."""
        out = []
        for it in self.plan[k]:
            mod = self.enc.aspp if it == "aspp" else (self.enc.backbone if it == "stem" else it)
            if it == "stem":
                out += [mod.conv1.weight, mod.bn1.weight, mod.bn1.bias]
            else:
                out += [p for p in mod.parameters() if p.requires_grad]
        return out

    def stash(self, rec, dfa):
        self.rec, self.dfa = rec, dfa

    def run(self, k):
        rec, grads = self.rec, GradSink(self.arena)
        by_blk = {it[1]: it for it in rec[1:-1]}
        f8 = getattr(self.enc, "_cn_fp8", None)
        if f8 is not None and k == 0:
            f8.grads.begin()
        wq = WgradQueue()     # the segment's weight gradients, grouped at its end (its bucket)
        for it in self.plan[k]:
            if it == "aspp":
                self.dx = aspp_bwd(rec[-1], self.dfa, grads)
            elif it == "stem":
                stem_bwd(rec[0], self.dx, grads)
            else:
                self.dx = bottleneck_bwd(by_blk[it], self.dx, grads, wq=wq)
        wq.flush()
        if k == len(self.plan) - 1:
            self.rec = self.dfa = self.dx = None
            if f8 is not None:
                f8.grads.end()
        return grads


def encode_pair(enc, img_a, img_b):
    """(features of frame a, features of frame b, (n, h, w)) for one encoder."""
    params = list(enc.parameters())
    fa, fb = EncoderPairFn.apply(img_a, img_b, enc, *params)
    n = img_a.shape[0]
    h, w = img_a.shape[2], img_a.shape[3]
    oh, ow = ops.out_hw(h, w, 7, 2, 3, 1)
    ph, pw = ops.pool_out(oh), ops.pool_out(ow)
    fh, fw = ops.out_hw(ph, pw, 1, 2, 0, 1)  # layer2 stride 2; layers 3-4 keep the size
    return fa, fb, (n, fh, fw)
