"""Tensor-level wrappers over the C ABI (no autograd here).

Activations are 2-D tensors [P, C] = NHWC flattened, possibly a channel-slice view of a
wider buffer (row stride = t.stride(0)).  Every function launches HIP kernels from
libcosnet_hip on the current torch stream; nothing here computes with torch ops.
"""
import weakref

import torch

from . import _native as nv

BN_EPS = 1e-5
BN_MOMENTUM = 0.1


def ld(t):
    assert t.dim() == 2 and t.stride(1) == 1, "expected a row-major 2-D [P, C] view"
    return t.stride(0)


def dtc(t):
    return nv.dtype_code(t.dtype)


def out_hw(h, w, k, s, p, d):
    return (h + 2 * p - d * (k - 1) - 1) // s + 1, (w + 2 * p - d * (k - 1) - 1) // s + 1


def pool_out(h, k=3, s=2, p=1):
    """MaxPool2d output size with ceil_mode=True (deeplab/residual_net.py:109)."""
    o = -(-(h + 2 * p - (k - 1) - 1) // s) + 1
    if (o - 1) * s >= h + p:
        o -= 1
    return o


# ---- optional per-launch timing of the implicit-GEMM kernel (bench.py roofline) -----------
class GemmProfile:
    """Records (algorithmic FLOPs, start, end) HIP events around every implicit-GEMM launch
    on the current stream while active."""

    active = None

    def __init__(self):
        self.rec = []

    def __enter__(self):
        GemmProfile.active = self
        return self

    def __exit__(self, *a):
        GemmProfile.active = None
        return False

    def summary(self):
        """(launches, total FLOPs, total kernel seconds) — call after synchronize()."""
        fl = sum(r[0] for r in self.rec)
        t = sum(r[1].elapsed_time(r[2]) for r in self.rec) * 1e-3
        return len(self.rec), fl, t

    def algorithmic_bytes(self):
        """Total unique operand bytes of the recorded launches: each GEMM's inputs read once
        (the conv input tensor itself, not its implicit im2col) plus its output written once."""
        return sum(r[4] for r in self.rec)

    def select(self, op):
        """(launches, FLOPs, seconds, algorithmic bytes) of the launches whose tag op == `op`."""
        sel = [r for r in self.rec if r[3] is not None and r[3][0] == op]
        return (len(sel), sum(r[0] for r in sel),
                sum(r[1].elapsed_time(r[2]) for r in sel) * 1e-3, sum(r[4] for r in sel))

    def by_tag(self):
        """{tag: [launches, FLOPs, seconds]} -- tag = (op, M, N, K) of each launch."""
        out = {}
        for fl, e0, e1, tag, _ in self.rec:
            r = out.setdefault(tag, [0, 0.0, 0.0])
            r[0] += 1
            r[1] += fl
            r[2] += e0.elapsed_time(e1) * 1e-3
        return out


def _prof_start(flops, tag=None, nbytes=0):
    p = GemmProfile.active
    if p is None:
        return None
    if torch.cuda.is_current_stream_capturing():
        return None  # ROCm has no timing event nodes in graphs: profile an eager step instead
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    p.rec.append((flops, e0, e1, tag, nbytes))
    return e1


def _prof_end(e1):
    if e1 is not None:
        e1.record()


# ---- weights -------------------------------------------------------------------------------
class WeightCache:
    """Compute-dtype copies of fp32 master conv weights: [Cout][KH][KW][Cp] for the forward
    GEMM and [Cin][KH][KW][Cout] for dgrad.

    One entry per (parameter, dtype, cin padding), with storage that is allocated once and
    never replaced (a recorded HIP graph keeps reading it).  An entry is valid while its tag
    (torch version counter, `epoch`, data pointer) matches; a stale entry is re-prepared IN
    PLACE.  The SGD kernel rewrites the copies of every parameter it updates in the same
    pass (optim.SGD, cn_sgd) and re-validates the entry (`refreshed`), so a training step
    runs no separate preparation kernels.  Bumping `epoch` invalidates everything."""

    epoch = 0

    def __init__(self):
        self._c = {}

    @staticmethod
    def _tag(w):
        return (w._version, WeightCache.epoch, w.data_ptr())

    def get(self, w, dtype, cin_pad=None, need_t=True):
        key = (id(w), tuple(w.shape), dtype, cin_pad)
        hit = self._c.get(key)
        if hit is not None and hit[0] == self._tag(w) and (hit[2] is not None or not need_t):
            return hit[1], hit[2]
        cout = w.shape[0]
        cin = w.shape[1]
        khw = w.shape[2] * w.shape[3] if w.dim() == 4 else 1
        cp = cin_pad or cin
        if w.dim() == 4:
            assert w.is_contiguous(memory_format=torch.channels_last), "conv weight must be channels_last"
        if hit is None:
            wf = torch.empty((cout, khw * cp), dtype=dtype, device=w.device)
            wt = torch.empty((cin, khw * cout), dtype=dtype, device=w.device) if need_t else None
            hit = [None, wf, wt, weakref.ref(w, lambda _r, k=key: self._c.pop(k, None))]
            self._c[key] = hit
        elif need_t and hit[2] is None:
            hit[2] = torch.empty((cin, khw * cout), dtype=dtype, device=w.device)
        nv.call("cn_weight_prep", nv.dtype_code(dtype), w.data_ptr(), cout, khw, cin, cp,
                hit[1].data_ptr(), nv.ptr(hit[2]), nv.stream())
        hit[0] = self._tag(w)
        return hit[1], hit[2]

    def entries(self, w):
        """[(wf, wt_or_None, cout, khw, cin, cp, entry)] of parameter w."""
        out = []
        for key, e in self._c.items():
            if key[0] == id(w) and e[3]() is w:
                cout, cin = w.shape[0], w.shape[1]
                khw = w.shape[2] * w.shape[3] if w.dim() == 4 else 1
                out.append((e[1], e[2], cout, khw, cin, e[1].shape[1] // khw, e))
        return out

    def refreshed(self, entry):
        """The SGD kernel rewrote this entry from the updated master weights."""
        w = entry[3]()
        entry[0] = self._tag(w) if w is not None else None

    @staticmethod
    def invalidate(entry):
        entry[0] = None


WCACHE = WeightCache()


# ---- convolution ----------------------------------------------------------------------------
def conv_fwd(x, n, h, w, wf, cout, k, stride, pad, dil, bias=None, out=None):
    """x [n*h*w, >=cin] -> y [n*oh*ow, cout] (or written into `out`)."""
    cin = wf.shape[1] // (k * k)
    oh, ow = out_hw(h, w, k, stride, pad, dil)
    if out is None:
        out = torch.empty((n * oh * ow, cout), dtype=x.dtype, device=x.device)
    es = x.element_size()
    ev = _prof_start(2.0 * n * oh * ow * cout * k * k * cin, ("fwd", n * oh * ow, cout, k * k * cin),
                     es * (n * h * w * cin + cout * k * k * cin + n * oh * ow * cout))
    nws = fwd_split_floats(x, n * oh * ow, cout, k * k * cin)
    if nws:   # deep one-round conv (the ASPP bottleneck): 256x256 tiles split over K
        ws = torch.empty((nws,), dtype=torch.float32, device=x.device)
        nv.call("cn_conv_fwd_ws", dtc(x), x.data_ptr(), ld(x), n, h, w, cin, wf.data_ptr(), cout, k,
                k, stride, pad, dil, nv.ptr(bias), out.data_ptr(), ld(out), oh, ow, ws.data_ptr(),
                nws, nv.stream())
    else:
        nv.call("cn_conv_fwd", dtc(x), x.data_ptr(), ld(x), n, h, w, cin, wf.data_ptr(), cout, k, k,
                stride, pad, dil, nv.ptr(bias), out.data_ptr(), ld(out), oh, ow, nv.stream())
    _prof_end(ev)
    return out, oh, ow


def fwd_split_floats(x, m, cout, kdim):
    """Workspace of the split-K forward (cn_conv_fwd_workspace_floats; 0: the shape does not split)."""
    return int(nv.query("cn_conv_fwd_workspace_floats", dtc(x), m, cout, kdim))


def conv_fwd_bn(x, n, h, w, wf, cout, k, stride, pad, dil, bn, nseg=1, bias=None):
    """Train mode: y = conv(x) (+ bias) and the BN batch statistics of y from the GEMM epilogue
    (cn_conv_fwd_bn: no pass of its own over y).  Returns (y, oh, ow, (mean, invstd)) with
    [nseg*cout] statistics; bn.running_* updated once per segment like bn_stats."""
    cin = wf.shape[1] // (k * k)
    oh, ow = out_hw(h, w, k, stride, pad, dil)
    M = n * oh * ow
    if M % nseg or M // nseg <= 1:
        raise ValueError("Expected more than 1 value per channel when training, got input size "
                         "torch.Size([%d, %d, 1, 1])" % (M // nseg, cout))
    if fwd_split_floats(x, M, cout, k * k * cin):
        # split over K: the statistics come from their own pass over the reduced output
        y, oh, ow = conv_fwd(x, n, h, w, wf, cout, k, stride, pad, dil, bias=bias)
        return y, oh, ow, bn_stats(y, bn, True, nseg)
    out = torch.empty((M, cout), dtype=x.dtype, device=x.device)
    mean = torch.empty((nseg * cout,), dtype=torch.float32, device=x.device)
    invstd = torch.empty_like(mean)
    nws = int(nv.query("cn_conv_fwd_bn_workspace_floats", dtc(x), M, cout, k * k * cin))
    ws = torch.empty((nws,), dtype=torch.float32, device=x.device)
    es = x.element_size()
    ev = _prof_start(2.0 * M * cout * k * k * cin, ("fwd", M, cout, k * k * cin),
                     es * (n * h * w * cin + cout * k * k * cin + M * cout))
    mom = bn.momentum if bn.momentum is not None else BN_MOMENTUM
    nv.call("cn_conv_fwd_bn", dtc(x), x.data_ptr(), ld(x), n, h, w, cin, wf.data_ptr(), cout, k, k,
            stride, pad, dil, nv.ptr(bias), out.data_ptr(), ld(out), oh, ow, nseg, ws.data_ptr(),
            mean.data_ptr(), invstd.data_ptr(), bn.running_mean.data_ptr(), bn.running_var.data_ptr(),
            float(mom), float(bn.eps), nv.stream())
    _prof_end(ev)
    bn._cn_nbt = getattr(bn, "_cn_nbt", 0) + nseg
    return out, oh, ow, (mean, invstd)


def conv_dgrad_bn(dy, n, oh, ow, wt, cin, k, pad, dil, x, stats, bn, dgamma=None, dbeta=None):
    """Stride-1 conv input-gradient fused with the backward reduction of the BN + ReLU whose
    pre-activation x [n*oh*ow, cin] fed the conv (cn_conv_dgrad_bn).  Returns
    (dy_bn [P, cin], dgamma, dbeta): the gradient at the BN output and the BN's parameter
    gradients (= the sums cn_bn_bwd_apply needs)."""
    cout = wt.shape[1] // (k * k)
    P = n * oh * ow
    out = torch.empty((P, cin), dtype=dy.dtype, device=dy.device)
    if dgamma is None:
        dgamma = torch.empty((cin,), dtype=torch.float32, device=dy.device)
    if dbeta is None:
        dbeta = torch.empty((cin,), dtype=torch.float32, device=dy.device)
    nws = int(nv.query("cn_conv_dgrad_bn_workspace_floats", dtc(dy), P, cin, k * k * cout))
    ws = torch.empty((nws,), dtype=torch.float32, device=dy.device)
    es = dy.element_size()
    ev = _prof_start(2.0 * P * cout * k * k * cin, ("dgrad1", P, cin, k * k * cout),
                     es * (P * cout + cout * k * k * cin + 2 * P * cin))
    g, b = _affine(bn)
    nv.call("cn_conv_dgrad_bn", dtc(dy), dy.data_ptr(), ld(dy), n, oh, ow, cout, wt.data_ptr(), cin,
            k, k, pad, dil, out.data_ptr(), ld(out), oh, ow, x.data_ptr(), ld(x),
            stats[0].data_ptr(), stats[1].data_ptr(), nv.ptr(g), nv.ptr(b), dbeta.data_ptr(),
            dgamma.data_ptr(), ws.data_ptr(), nv.stream())
    _prof_end(ev)
    return out, dgamma, dbeta


def bn_bwd_apply(x, dy, stats, bn, dgamma, dbeta, out=None):
    """dx of a train-mode BN + ReLU (mask from x) given its parameter-gradient sums."""
    p, c = x.shape
    if out is None:
        out = torch.empty((p, c), dtype=x.dtype, device=x.device)
    g, b = _affine(bn)
    nv.call("cn_bn_bwd_apply", dtc(x), x.data_ptr(), ld(x), dy.data_ptr(), ld(dy), p, c,
            stats[0].data_ptr(), stats[1].data_ptr(), nv.ptr(g), nv.ptr(b), dbeta.data_ptr(),
            dgamma.data_ptr(), out.data_ptr(), ld(out), nv.stream())
    return out


# ---- fp8 (e4m3) operands (BASELINE configs[4]) ------------------------------------------------
FP8_E4M3, FP8_E5M2 = 0, 1
FMT_MAX = {FP8_E4M3: 448.0, FP8_E5M2: 57344.0}


def fp8_state(device, fmt=FP8_E4M3):
    """Per-tensor fp8 scaling state [scale, 1/scale, amax, format max] (cn_fp8_quant_fmt)."""
    return torch.tensor([1.0, 1.0, 0.0, FMT_MAX[fmt]], dtype=torch.float32, device=device)


FP8_DELAYED, FP8_CURRENT, FP8_AMAX = 0, 1, 2


def fp8_quant(x, state, mode=FP8_CURRENT, out=None, fmt=FP8_E4M3):
    """x [P, C] (fp32 / bf16) -> fp8 bytes [P, C] (uint8; e4m3, or e5m2 with fmt=FP8_E5M2)
    scaled by state (see fp8_state)."""
    p, c = x.shape
    if out is None and mode != FP8_AMAX:
        out = torch.empty((p, c), dtype=torch.uint8, device=x.device)
    nv.call("cn_fp8_quant_fmt", dtc(x), fmt, x.data_ptr(), ld(x), p, c, nv.ptr(out),
            ld(out) if out is not None else c, state.data_ptr(), mode, nv.stream())
    return out


def fp8_update(states, margin=1.0):
    """Turn each state's collected amax into its next scale (states: [n, 4] or [4])."""
    nv.call("cn_fp8_update", states.data_ptr(), states.numel() // 4, float(margin), nv.stream())


def conv_dgrad_fp8(dy8, n, oh, ow, wt8, cin, k, pad, dil, h, w, dy_state, w_state, out=None,
                   accumulate=False):
    """dx (bf16) (+)= conv_dgrad(dy8 e5m2, wt8 e4m3) * s_dy * s_w, stride 1 (fp8 mode)."""
    cout = wt8.shape[1] // (k * k)
    if out is None:
        out = torch.empty((n * h * w, cin), dtype=torch.bfloat16, device=dy8.device)
    ev = _prof_start(2.0 * n * h * w * cin * k * k * cout, ("dgrad8", n * h * w, cin, k * k * cout),
                     n * oh * ow * cout + cin * k * k * cout + 2 * n * h * w * cin)
    nv.call("cn_conv_dgrad_fp8", dy8.data_ptr(), ld(dy8), n, oh, ow, cout, wt8.data_ptr(), cin, k, k,
            pad, dil, out.data_ptr(), ld(out), h, w, int(accumulate), dy_state.data_ptr(),
            w_state.data_ptr(), nv.stream())
    _prof_end(ev)
    return out


def conv_fwd_fp8(x8, n, h, w, wf8, cout, k, stride, pad, dil, x_state, w_state, bias=None,
                 out=None):
    """y (bf16) = conv(x8, w8) * sx * sw (+ bias): the fp8 implicit-GEMM conv."""
    cin = wf8.shape[1] // (k * k)
    oh, ow = out_hw(h, w, k, stride, pad, dil)
    if out is None:
        out = torch.empty((n * oh * ow, cout), dtype=torch.bfloat16, device=x8.device)
    ev = _prof_start(2.0 * n * oh * ow * cout * k * k * cin, ("fwd8", n * oh * ow, cout, k * k * cin),
                     n * h * w * cin + cout * k * k * cin + 2 * n * oh * ow * cout)
    nv.call("cn_conv_fwd_fp8", x8.data_ptr(), ld(x8), n, h, w, cin, wf8.data_ptr(), cout, k, k,
            stride, pad, dil, nv.ptr(bias), out.data_ptr(), ld(out), oh, ow, x_state.data_ptr(),
            w_state.data_ptr(), nv.stream())
    _prof_end(ev)
    return out, oh, ow


def conv_fwd_bn_grouped(x, n, h, w, wfs, cout, k, dils, bns, nseg=1, biases=None):
    """The ASPP's atrous branches as ONE grouped launch (cn_conv_fwd_bn_grouped): for each g,
    y_g = conv(x, wfs[g], dilation dils[g], padding dils[g]) (+ biases[g]) and the BN batch
    statistics of y_g from the GEMM epilogue (as conv_fwd_bn).  Returns [(y_g, (mean, invstd))]."""
    import ctypes
    G = len(wfs)
    cin = wfs[0].shape[1] // (k * k)
    M = n * h * w
    if M % nseg or M // nseg <= 1:
        raise ValueError("Expected more than 1 value per channel when training, got input size "
                         "torch.Size([%d, %d, 1, 1])" % (M // nseg, cout))
    dev = x.device
    ys = [torch.empty((M, cout), dtype=x.dtype, device=dev) for _ in range(G)]
    means = [torch.empty((nseg * cout,), dtype=torch.float32, device=dev) for _ in range(G)]
    invs = [torch.empty_like(m) for m in means]
    nws = int(nv.query("cn_conv_fwd_bn_workspace_floats", dtc(x), M, cout, k * k * cin))
    wss = [torch.empty((nws,), dtype=torch.float32, device=dev) for _ in range(G)]
    biases = biases or [None] * G
    P = lambda ts: (ctypes.c_void_p * G)(*[t.data_ptr() if t is not None else None for t in ts])
    es = x.element_size()
    ev = _prof_start(2.0 * G * M * cout * k * k * cin, ("fwd", M, cout * G, k * k * cin),
                     es * (n * h * w * cin + G * cout * k * k * cin + G * M * cout))
    mom = bns[0].momentum if bns[0].momentum is not None else BN_MOMENTUM
    nv.call("cn_conv_fwd_bn_grouped", dtc(x), x.data_ptr(), ld(x), n, h, w, cin, G, P(wfs), cout, k, k,
            (ctypes.c_int * G)(*dils), P(biases), P(ys), cout, nseg, P(wss), P(means), P(invs),
            P([b.running_mean for b in bns]), P([b.running_var for b in bns]), float(mom),
            float(bns[0].eps), nv.stream())
    _prof_end(ev)
    for b in bns:
        b._cn_nbt = getattr(b, "_cn_nbt", 0) + nseg
    return [(y, (m, i)) for y, m, i in zip(ys, means, invs)]


def conv_fwd_fp8_bn(x8, n, h, w, wf8, cout, k, stride, pad, dil, x_state, w_state, bn, nseg=1,
                    bias=None):
    """conv_fwd_fp8 + the BN batch statistics of its stored bf16 output from the GEMM epilogue
    (cn_conv_fwd_fp8_bn), as conv_fwd_bn does for bf16.  Returns (y, oh, ow, (mean, invstd))."""
    cin = wf8.shape[1] // (k * k)
    oh, ow = out_hw(h, w, k, stride, pad, dil)
    M = n * oh * ow
    if M % nseg or M // nseg <= 1:
        raise ValueError("Expected more than 1 value per channel when training, got input size "
                         "torch.Size([%d, %d, 1, 1])" % (M // nseg, cout))
    out = torch.empty((M, cout), dtype=torch.bfloat16, device=x8.device)
    mean = torch.empty((nseg * cout,), dtype=torch.float32, device=x8.device)
    invstd = torch.empty_like(mean)
    nws = int(nv.query("cn_conv_fwd_bn_workspace_floats", 2, M, cout, k * k * cin))
    ws = torch.empty((nws,), dtype=torch.float32, device=x8.device)
    ev = _prof_start(2.0 * M * cout * k * k * cin, ("fwd8", M, cout, k * k * cin),
                     n * h * w * cin + cout * k * k * cin + 2 * M * cout)
    mom = bn.momentum if bn.momentum is not None else BN_MOMENTUM
    nv.call("cn_conv_fwd_fp8_bn", x8.data_ptr(), ld(x8), n, h, w, cin, wf8.data_ptr(), cout, k, k,
            stride, pad, dil, nv.ptr(bias), out.data_ptr(), ld(out), oh, ow, x_state.data_ptr(),
            w_state.data_ptr(), nseg, ws.data_ptr(), mean.data_ptr(), invstd.data_ptr(),
            bn.running_mean.data_ptr(), bn.running_var.data_ptr(), float(mom), float(bn.eps),
            nv.stream())
    _prof_end(ev)
    bn._cn_nbt = getattr(bn, "_cn_nbt", 0) + nseg
    return out, oh, ow, (mean, invstd)


def conv_dgrad(dy, n, oh, ow, wt, cin, k, stride, pad, dil, h, w, out=None, accumulate=False):
    cout = wt.shape[1] // (k * k)
    if out is None:
        out = torch.empty((n * h * w, cin), dtype=dy.dtype, device=dy.device)
    es = dy.element_size()
    ev = _prof_start(2.0 * n * oh * ow * cout * k * k * cin, ("dgrad%d" % stride, n * h * w, cin, k * k * cout),
                     es * (n * oh * ow * cout + cout * k * k * cin + n * h * w * cin))
    nv.call("cn_conv_dgrad", dtc(dy), dy.data_ptr(), ld(dy), n, oh, ow, cout, wt.data_ptr(), cin,
            k, k, stride, pad, dil, out.data_ptr(), ld(out), h, w, int(accumulate), nv.stream())
    _prof_end(ev)
    return out


def conv_wgrad(x, n, h, w, cin, dy, oh, ow, cout, k, stride, pad, dil, dw=None):
    """fp32 [cout, k*k*cin] weight gradient (channels_last order), fully overwritten."""
    if dw is None:
        dw = torch.empty((cout, k * k * cin), dtype=torch.float32, device=x.device)
    nws = int(nv.query("cn_conv_wgrad_workspace_floats", dtc(x), n, oh, ow, cout, k, k, cin))
    ws = torch.empty((nws,), dtype=torch.float32, device=x.device) if nws else None
    es = x.element_size()
    ev = _prof_start(2.0 * n * oh * ow * cout * k * k * cin, ("wgrad", cout, k * k * cin, n * oh * ow),
                     es * (n * h * w * cin + n * oh * ow * cout) + 4 * cout * k * k * cin)
    nv.call("cn_conv_wgrad", dtc(x), x.data_ptr(), ld(x), n, h, w, cin, dy.data_ptr(), ld(dy), oh,
            ow, cout, k, k, stride, pad, dil, dw.data_ptr(), nv.ptr(ws), nv.stream())
    _prof_end(ev)
    return dw


GROUP_MAX = 24       # cn_conv_wgrad_grouped's problem limit (gemm.h GEMM_MAXG)


def conv_wgrad_grouped(jobs, n, h, w, cin, oh, ow, cout, k, stride, pad, dil, split=False):
    """Weight gradients of G convs of ONE shape in one launch (cn_conv_wgrad_grouped): jobs =
    [(x, dy, dw)] with x [n*h*w, cin], dy [n*oh*ow, cout] sharing the row strides, dw fp32
    [cout, k*k*cin] (written).  No split-K workspace and no reduce launch.  split=True: the G
    problems also split over K (cn_conv_wgrad_grouped_ws: one GEMM launch + one reduce launch
    for the group), for shapes too small to fill the chip grouped whole."""
    import ctypes
    g = len(jobs)
    if not 1 <= g <= GROUP_MAX:
        raise ValueError("1..%d problems per grouped launch" % GROUP_MAX)
    x0, dy0, _ = jobs[0]
    if any(ld(x) != ld(x0) or ld(dy) != ld(dy0) for x, dy, _ in jobs):
        raise ValueError("grouped weight gradients need equal row strides")
    xs = (ctypes.c_void_p * g)(*[x.data_ptr() for x, _, _ in jobs])
    dys = (ctypes.c_void_p * g)(*[dy.data_ptr() for _, dy, _ in jobs])
    dws = (ctypes.c_void_p * g)(*[dw.data_ptr() for _, _, dw in jobs])
    es = x0.element_size()
    fl = 2.0 * n * oh * ow * cout * k * k * cin
    ev = _prof_start(g * fl, ("wgrad", cout, k * k * cin, n * oh * ow),
                     g * (es * (n * h * w * cin + n * oh * ow * cout) + 4 * cout * k * k * cin))
    nws = int(nv.query("cn_conv_wgrad_grouped_workspace_floats", dtc(x0), g, n, oh, ow, cout, k, k,
                       cin)) if split else 0
    if nws:
        ws = torch.empty((nws,), dtype=torch.float32, device=x0.device)
        nv.call("cn_conv_wgrad_grouped_ws", dtc(x0), g, ctypes.addressof(xs), ld(x0), n, h, w, cin,
                ctypes.addressof(dys), ld(dy0), oh, ow, cout, k, k, stride, pad, dil,
                ctypes.addressof(dws), ws.data_ptr(), nws, nv.stream())
    else:
        nv.call("cn_conv_wgrad_grouped", dtc(x0), g, ctypes.addressof(xs), ld(x0), n, h, w, cin,
                ctypes.addressof(dys), ld(dy0), oh, ow, cout, k, k, stride, pad, dil,
                ctypes.addressof(dws), nv.stream())
    _prof_end(ev)
    return [dw for _, _, dw in jobs]


def conv_wgrad_fp8(jobs, n, h, w, cin, oh, ow, cout, k, stride, pad, dil):
    """fp8 weight gradients of G <= GROUP_MAX convs of ONE shape in one launch (cn_conv_wgrad_fp8,
    BASELINE configs[4]): jobs = [(x8, x_state, dy8, dy_state, dw)] with x8 e4m3 [n*h*w, cin] (the
    fp8 forward conv's input copy), dy8 e5m2 [n*oh*ow, cout] (the fp8 dgrad's output-gradient
    copy), their [4]-float scale states (element 0 = dequantisation scale) and dw fp32
    [cout, k*k*cin] (written).  Split over K into slabs + one reduce launch when small."""
    import ctypes
    g = len(jobs)
    if not 1 <= g <= GROUP_MAX:
        raise ValueError("1..%d problems per grouped launch" % GROUP_MAX)
    x0, _, d0, _, _ = jobs[0]
    if any(ld(x) != ld(x0) or ld(dy) != ld(d0) for x, _, dy, _, _ in jobs):
        raise ValueError("grouped weight gradients need equal row strides")
    arr = lambda vals: (ctypes.c_void_p * g)(*vals)
    xs = arr([j[0].data_ptr() for j in jobs])
    xst = arr([j[1].data_ptr() for j in jobs])
    dys = arr([j[2].data_ptr() for j in jobs])
    dst = arr([j[3].data_ptr() for j in jobs])
    dws = arr([j[4].data_ptr() for j in jobs])
    fl = 2.0 * n * oh * ow * cout * k * k * cin
    ev = _prof_start(g * fl, ("wgrad8", cout, k * k * cin, n * oh * ow),
                     g * ((n * h * w * cin + n * oh * ow * cout) + 4 * cout * k * k * cin))
    nws = int(nv.query("cn_conv_wgrad_fp8_workspace_floats", g, n, oh, ow, cout, k, k, cin))
    ws = torch.empty((nws,), dtype=torch.float32, device=x0.device) if nws else None
    nv.call("cn_conv_wgrad_fp8", g, ctypes.addressof(xs), ld(x0), n, h, w, cin, ctypes.addressof(dys),
            ld(d0), oh, ow, cout, k, k, stride, pad, dil, ctypes.addressof(dws), ctypes.addressof(xst),
            ctypes.addressof(dst), nv.ptr(ws), nws, nv.stream())
    _prof_end(ev)
    return [j[4] for j in jobs]


def as_param_grad(dw_flat, weight):
    """[cout, k*k*cin] fp32 (OHWI order) -> gradient shaped/stided like the channels_last param."""
    if weight.dim() == 2:
        return dw_flat.view(weight.shape)
    co, ci, kh, kw = weight.shape
    return dw_flat.view(co, kh, kw, ci).permute(0, 3, 1, 2)


def colpart_ws(p, c, device):
    """Workspace of the deterministic column reductions (colsum, gate / head backward)."""
    n = int(nv.query("cn_colpart_workspace_floats", p, c))
    return torch.empty((max(n, 1),), dtype=torch.float32, device=device)


def colsum(x, out=None):
    """fp32 [C] column sums of x [P, C] (bias gradients), fixed-order (bitwise repeatable)."""
    if out is None:
        out = torch.empty((x.shape[1],), dtype=torch.float32, device=x.device)
    ws = colpart_ws(x.shape[0], x.shape[1], x.device)
    nv.call("cn_colsum", dtc(x), x.data_ptr(), ld(x), x.shape[0], x.shape[1], out.data_ptr(),
            ws.data_ptr(), nv.stream())
    return out


def avgpool(x, n, hw, scale, out):
    """out [n, C] = scale * sum over the hw rows of each image of x [n*hw, C] (C = out width);
    deterministic fixed-order reduction of row-split partials (AdaptiveAvgPool2d(1),
    deeplab/deeplabv3_encoder.py:57; and its backward with scale 1)."""
    c = out.shape[1]
    nws = int(nv.query("cn_avgpool_workspace_floats", dtc(x), n, hw, c))
    ws = torch.empty((max(nws, 1),), dtype=torch.float32, device=x.device)
    nv.call("cn_avgpool", dtc(x), x.data_ptr(), ld(x), n, hw, c, float(scale), out.data_ptr(),
            ws.data_ptr(), nv.stream())
    return out


GEMM_KC, GEMM_MC = 0, 2


def gemm(a, b, m, n, k, layout_a=GEMM_KC, layout_b=GEMM_KC, lda=None, ldb=None, a_bs=0, b_bs=0,
         out=None, ldc=None, c_bs=0, c_mode=0, batch=1, ka_lim=None, kb_lim=None, out_dtype=None,
         nsplit=1, alpha=1.0, bias=None, tag=None):
    """C[m, n] = alpha * sum_k A[m, k] * B[n, k] (batched via *_bs element strides)."""
    dt = a.dtype
    if out is None:
        out = torch.empty((batch * m, n), dtype=out_dtype or dt, device=a.device)
        ldc = n
        c_bs = m * n
    c_f32 = int(out.dtype == torch.float32)
    ev = _prof_start(2.0 * batch * m * n * (kb_lim if kb_lim is not None else k),
                     (tag or "gemm%d%d" % (layout_a, layout_b), batch * m, n, k),
                     (batch if a_bs else 1) * m * k * a.element_size() +
                     (batch if b_bs else 1) * n * k * b.element_size() +
                     batch * m * n * out.element_size())
    if nsplit > 1 and c_mode in (0, 1) and batch == 1 and c_f32 and ldc == n:
        # split-K into fp32 slabs + fixed-order reduction (no atomic contention)
        slab = m * n
        ws = torch.empty((nsplit * slab,), dtype=torch.float32, device=a.device)
        nv.call("cn_gemm", nv.dtype_code(dt), layout_a, layout_b, m, n, k,
                k if ka_lim is None else ka_lim, k if kb_lim is None else kb_lim,
                a.data_ptr(), lda, a_bs, b.data_ptr(), ldb, b_bs, ws.data_ptr(), ldc, 0, 1,
                3, float(alpha), None, 1, nsplit, slab, nv.stream())
        nv.call("cn_splitk_reduce", ws.data_ptr(), _nsplit_eff(k, nsplit, dt), slab, slab,
                out.data_ptr(), int(c_mode == 1), nv.stream())
    else:
        nv.call("cn_gemm", nv.dtype_code(dt), layout_a, layout_b, m, n, k,
                k if ka_lim is None else ka_lim, k if kb_lim is None else kb_lim,
                a.data_ptr(), lda, a_bs, b.data_ptr(), ldb, b_bs, out.data_ptr(), ldc, c_bs, c_f32,
                c_mode, float(alpha), nv.ptr(bias), batch, nsplit, 0, nv.stream())
    _prof_end(ev)
    return out


# ---- fused co-attention (inference) ----------------------------------------------------------
import os as _os

# COSNET_COATT_FUSED=0 keeps the materialised-S path for inference too (A/B, tests)
COATT_FUSED = _os.environ.get("COSNET_COATT_FUSED", "1") != "0"


def coatt_fused_ok(dt, c, va, vb):
    """The fused kernel covers bf16, C = 256 and 16-byte aligned rows (every RAA call site)."""
    return (COATT_FUSED and dt == torch.bfloat16 and c == 256 and ld(va) % 8 == 0
            and ld(vb) % 8 == 0 and va.data_ptr() % 16 == 0 and vb.data_ptr() % 16 == 0)


def coatt_fused(vat, va, vb, n, hw, za=None, zb=None):
    """Z_a = softmax_j(S) Vb and Z_b = softmax_i(S)^T Va with S = vat vb^T, never materialised
    (rgbd_segmentation_RAA.py:160-170).  Algorithmic work: 3 x 2 HW^2 C per pair."""
    c = vat.shape[1]
    ev = _prof_start(3 * 2.0 * n * hw * hw * c, ("coatt_fused", n, hw, c),
                     (3 * n * hw * c + 2 * n * hw * c) * vat.element_size())
    ndir = (za is not None) + (zb is not None)
    nws = int(nv.query("cn_coatt_fused_workspace_bytes", n, hw, ndir))
    ws = torch.empty((nws // 4,), dtype=torch.float32, device=vat.device) if nws else None
    nv.call("cn_coatt_fused_fwd_ws", vat.data_ptr(), ld(vat), va.data_ptr(), ld(va), vb.data_ptr(),
            ld(vb), n, hw, c, nv.ptr(za), nv.ptr(zb), ld(za if za is not None else zb), nv.ptr(ws),
            nws, nv.stream())
    _prof_end(ev)
    return za, zb


def hw_pad(hw):
    return (hw + 31) // 32 * 32


def coatt_f8(vat, va, vb, n, hw, za, zb, lse_a=None, lse_b=None):
    """Both co-attention directions with MX-fp8 operands (BASELINE configs[4]: e4m3 bytes + one
    E8M0 exponent per 32 reduction values, the block-scaled 32x32x64 MFMA), softmax statistics
    in fp32; optional per-row log2-sum-exp2 [n, hw_pad(hw)] for the bf16 flash backward."""
    c = vat.shape[1]
    ev = _prof_start(3 * 2.0 * n * hw * hw * c, ("coatt_f8_fwd", n, hw, c),
                     (3 * n * hw * c + 2 * n * hw * c) * vat.element_size())
    nws = int(nv.query("cn_coatt_f8_workspace_bytes", n, hw))
    ws = torch.empty((nws,), dtype=torch.uint8, device=vat.device)
    nv.call("cn_coatt_f8_fwd", vat.data_ptr(), ld(vat), va.data_ptr(), ld(va), vb.data_ptr(), ld(vb),
            n, hw, c, za.data_ptr(), zb.data_ptr(), ld(za), nv.ptr(lse_a), nv.ptr(lse_b),
            ws.data_ptr(), nws, nv.stream())
    _prof_end(ev)
    return za, zb


def coatt_f8_train(vat, va, vb, n, hw, za, zb, lse_a, lse_b):
    """Training forward of both directions with MX-fp8 operands (configs[4]): Z_a, Z_b, the
    per-row log2-sum-exp2 normalisers, and the decoded operands (vat_q, va_q, vb_q) -- bf16,
    exact -- that the flash backward recomputes S and P from (cn_coatt_f8_train_fwd)."""
    c = vat.shape[1]
    ev = _prof_start(3 * 2.0 * n * hw * hw * c, ("coatt_f8_train_fwd", n, hw, c),
                     (3 * n * hw * c + 2 * n * hw * c) * vat.element_size())
    nws = int(nv.query("cn_coatt_f8_train_workspace_bytes", n, hw))
    ws = torch.empty((nws,), dtype=torch.uint8, device=vat.device)
    q = [torch.empty((n * hw, c), dtype=torch.bfloat16, device=vat.device) for _ in range(3)]
    nv.call("cn_coatt_f8_train_fwd", vat.data_ptr(), ld(vat), va.data_ptr(), ld(va), vb.data_ptr(),
            ld(vb), n, hw, c, za.data_ptr(), zb.data_ptr(), ld(za), lse_a.data_ptr(), lse_b.data_ptr(),
            q[0].data_ptr(), q[1].data_ptr(), q[2].data_ptr(), c, ws.data_ptr(), nws, nv.stream())
    _prof_end(ev)
    return tuple(q)


def coatt_flash_fwd(vat, va, vb, n, hw, za, zb, lse_a, lse_b):
    """Training forward of both co-attention directions (S never in HBM) + the per-row
    log2-sum-exp2 normalisers [n, hw_pad(hw)] the backward recomputes P from."""
    c = vat.shape[1]
    ev = _prof_start(3 * 2.0 * n * hw * hw * c, ("coatt_flash_fwd", n, hw, c),
                     (3 * n * hw * c + 2 * n * hw * c) * vat.element_size())
    nws = int(nv.query("cn_coatt_fused_workspace_bytes", n, hw, 2))
    ws = torch.empty((nws // 4,), dtype=torch.float32, device=vat.device) if nws else None
    nv.call("cn_coatt_flash_fwd_ws", vat.data_ptr(), ld(vat), va.data_ptr(), ld(va), vb.data_ptr(),
            ld(vb), n, hw, c, za.data_ptr(), zb.data_ptr(), ld(za), lse_a.data_ptr(),
            lse_b.data_ptr(), nv.ptr(ws), nws, nv.stream())
    _prof_end(ev)


def coatt_flash_bwd(vat, va, vb, wf, za, zb, lse_a, lse_b, dza, dzb, n, hw, dva=None,
                    dva_accumulate=False):
    """Backward of the flash co-attention: returns dVa_t [P, C] (bf16) and, if `dva` is given,
    accumulates dV_a's softmax-over-i term sum_j P1[i][j] dZ_b[j] into it.  Algorithmic work
    (the reference's autograd; the recomputed S is not counted): dP0 = dZa Vb^T
    and/or dP1 = Va dZb^T plus dVa_t = dS Vb in the dVa_t kernel, P1^T dZb in the PV kernel --
    4 x 2 HW^2 C per pair with both gradients, 2 with dZa only."""
    c = vat.shape[1]
    P = n * hw
    hwp = hw_pad(hw)
    dev = vat.device
    d0 = d1 = None
    if dza is not None:
        d0 = torch.empty((P,), dtype=torch.float32, device=dev)
        nv.call("cn_rowdot", dtc(dza), dza.data_ptr(), ld(dza), za.data_ptr(), ld(za), P, c,
                d0.data_ptr(), nv.stream())
    if dzb is not None:
        d1 = torch.empty((n * hwp,), dtype=torch.float32, device=dev)
        nv.call("cn_rowdot_seg", dtc(dzb), dzb.data_ptr(), ld(dzb), zb.data_ptr(), ld(zb), P, c, hw,
                hwp, d1.data_ptr(), nv.stream())
    dvat = torch.empty((P, c), dtype=vat.dtype, device=dev)
    nterm = (dza is not None) + (dzb is not None)
    ev = _prof_start((1 + nterm) * 2.0 * n * hw * hw * c, ("coatt_flash_bwd", n, hw, c),
                     (2 + 2 * nterm) * P * c * vat.element_size())
    # one workspace for the key-split partials of both kernels (they run one after the other)
    nws = max(int(nv.query("cn_coatt_flash_bwd_workspace_bytes", n, hw)),
              int(nv.query("cn_coatt_fused_workspace_bytes", n, hw, 1)) if dva is not None else 0)
    ws = torch.empty((nws // 4,), dtype=torch.float32, device=dev) if nws else None
    nv.call("cn_coatt_flash_dvat_ws", vat.data_ptr(), ld(vat), va.data_ptr(), ld(va), nv.ptr(dza),
            ld(dza) if dza is not None else c, vb.data_ptr(), ld(vb), nv.ptr(dzb),
            ld(dzb) if dzb is not None else c, lse_a.data_ptr(), nv.ptr(d0), lse_b.data_ptr(),
            nv.ptr(d1), n, hw, c, dvat.data_ptr(), ld(dvat), 0, nv.ptr(ws), nws, nv.stream())
    _prof_end(ev)
    if dva is not None and dzb is not None:
        ev = _prof_start(2.0 * n * hw * hw * c, ("coatt_flash_bwd", n, hw, c),
                         3 * P * c * vat.element_size())
        nv.call("cn_coatt_flash_pv_ws", vat.data_ptr(), ld(vat), vb.data_ptr(), ld(vb), dzb.data_ptr(),
                ld(dzb), lse_b.data_ptr(), n, hw, c, dva.data_ptr(), ld(dva), int(dva_accumulate),
                nv.ptr(ws), nws, nv.stream())
        _prof_end(ev)
    return dvat


def _nsplit_eff(k, nsplit, dt):
    """Number of splits cn_gemm really launches (chunks rounded up to whole K tiles)."""
    bk = 64 if dt == torch.bfloat16 else 32
    chunk = -(-k // nsplit)
    chunk = -(-chunk // bk) * bk
    return -(-k // chunk)


# ---- batch norm -------------------------------------------------------------------------------
def _ws(dtype, p, c, device, nseg=1):
    n = nv.query("cn_bn_workspace_floats", nv.dtype_code(dtype), p, c, nseg)
    return torch.empty((max(int(n), 1),), dtype=torch.float32, device=device)


def bn_stats(x, bn, training, nseg=1, count_update=True):
    """(mean, invstd) fp32 [nseg*C] of x = nseg stacked segments of equal rows, each its own
    BN batch (one reference BN call per frame).  Train mode updates bn.running_* once per
    segment, in order (momentum 0.1 each)."""
    p, c = x.shape
    if p % nseg:
        raise ValueError("rows %d not divisible into %d segments" % (p, nseg))
    p //= nseg
    mean = torch.empty((nseg * c,), dtype=torch.float32, device=x.device)
    invstd = torch.empty_like(mean)
    if training:
        if p <= 1:
            raise ValueError("Expected more than 1 value per channel when training, got input size "
                             "torch.Size([%d, %d, 1, 1])" % (p, c))
        ws = _ws(x.dtype, p, c, x.device, nseg)
        mom = bn.momentum if bn.momentum is not None else BN_MOMENTUM
        nv.call("cn_bn_stats", dtc(x), x.data_ptr(), ld(x), p, nseg, c, mean.data_ptr(),
                invstd.data_ptr(), bn.running_mean.data_ptr(), bn.running_var.data_ptr(), float(mom),
                float(bn.eps), ws.data_ptr(), nv.stream())
        if count_update:
            bn._cn_nbt = getattr(bn, "_cn_nbt", 0) + nseg
    else:
        nv.call("cn_bn_eval_params", bn.running_mean.data_ptr(), bn.running_var.data_ptr(), c,
                float(bn.eps), mean.data_ptr(), invstd.data_ptr(), nv.stream())
        if nseg > 1:
            mean[c:].view(nseg - 1, c).copy_(mean[:c].expand(nseg - 1, c))
            invstd[c:].view(nseg - 1, c).copy_(invstd[:c].expand(nseg - 1, c))
    return mean, invstd


def seg_of(stats, i, c):
    """Statistics of segment i out of bn_stats(..., nseg)."""
    return stats[0][i * c:(i + 1) * c], stats[1][i * c:(i + 1) * c]


def _affine(bn):
    if bn.affine:
        return bn.weight, bn.bias
    return None, None


def relu_mask(p, c, like):
    """Bit-mask buffer for bn_apply(mask=...): [p, c / vec] bytes (vec = channels per 16-B chunk)."""
    vec = 8 if like.dtype == torch.bfloat16 else 4
    return torch.empty((p, c // vec), dtype=torch.uint8, device=like.device)


def bn_apply(x, stats, bn, act=0, prelu=None, res=None, xr=None, rstats=None, rbn=None, out=None,
             nseg=1, out8=None, qstate=None, mask=None):
    """y = act(bn(x) [+ res] [+ rbn(xr)]) with per-segment statistics ([nseg*C] each); with
    out8 / qstate also an fp8 copy of y (delayed scaling, amax collected into qstate); with mask
    (relu_mask) also y > 0 as bits, which bn_bwd(act=4) takes instead of y."""
    p, c = x.shape
    if out is None:
        out = torch.empty((p, c), dtype=x.dtype, device=x.device)
    g, b = _affine(bn)
    rg, rb = _affine(rbn) if rbn is not None else (None, None)
    nv.call("cn_bn_apply_ex", dtc(x), x.data_ptr(), ld(x), p // nseg, nseg, c, stats[0].data_ptr(),
            stats[1].data_ptr(), nv.ptr(g), nv.ptr(b), nv.ptr(res), ld(res) if res is not None else 0,
            nv.ptr(xr), ld(xr) if xr is not None else 0, nv.ptr(rstats[0] if rstats else None),
            nv.ptr(rstats[1] if rstats else None), nv.ptr(rg), nv.ptr(rb), act, nv.ptr(prelu),
            out.data_ptr(), ld(out), nv.ptr(out8), ld(out8) if out8 is not None else 0,
            nv.ptr(qstate), nv.ptr(mask), mask.stride(0) if mask is not None else 0, nv.stream())
    return out


def bn_bwd(x, dy, y, stats, bn, act=0, prelu=None, want_dx=True, dx=None, dres=None, dgamma=None,
           dbeta=None, dprelu=None):
    """Train-mode BN backward (+ fused activation mask).  Returns dx, dgamma, dbeta, dprelu
    (dgamma / dbeta / dprelu written into the given buffers if any, e.g. gradient-arena slices).
    act=1 with y=None: the ReLU mask is recomputed from x with the forward's affine (no read of
    the activation; only valid when y = relu(bn(x)) had no residual added).  act=4: y is the
    bit mask bn_apply(mask=...) wrote (1/16 of y's bytes)."""
    p, c = x.shape
    if act == 1 and y is None:
        act = 3
    if dgamma is None:
        dgamma = torch.empty((c,), dtype=torch.float32, device=x.device)
    if dbeta is None:
        dbeta = torch.empty((c,), dtype=torch.float32, device=x.device)
    dpc = torch.empty((c,), dtype=torch.float32, device=x.device) if act == 2 else None
    if want_dx and dx is None:
        dx = torch.empty((p, c), dtype=x.dtype, device=x.device)
    ws = _ws(x.dtype, p, c, x.device)
    g, b = _affine(bn)
    nv.call("cn_bn_bwd", dtc(x), x.data_ptr(), ld(x), dy.data_ptr(), ld(dy), nv.ptr(y),
            (y.stride(0) if act == 4 else ld(y)) if y is not None else 0, p, c, stats[0].data_ptr(), stats[1].data_ptr(), nv.ptr(g),
            nv.ptr(b), act, nv.ptr(prelu), dgamma.data_ptr(), dbeta.data_ptr(), nv.ptr(dpc),
            nv.ptr(dx), ld(dx) if dx is not None else 0, nv.ptr(dres),
            ld(dres) if dres is not None else 0, ws.data_ptr(), nv.stream())
    if dpc is not None:  # per-channel partials -> the single PReLU weight (fixed order)
        if dprelu is None:
            dprelu = torch.empty((1,), dtype=torch.float32, device=x.device)
        nv.call("cn_sum_rows", dpc.data_ptr(), c, 1, dprelu.data_ptr(), nv.stream())
    return dx, dgamma, dbeta, dprelu


def cast_copy(src, dst, accumulate=False):
    nv.call("cn_cast2d", dtc(src), dtc(dst), src.data_ptr(), ld(src), src.shape[0], src.shape[1],
            dst.data_ptr(), ld(dst), int(accumulate), nv.stream())
    return dst
