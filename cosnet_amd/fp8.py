"""fp8 (OCP e4m3) forward convolutions: BASELINE configs[4] ("fp8 MFMA ... implicit-GEMM conv").

Recipe (the usual fp8-training split): the encoder convs' FORWARD GEMMs take e4m3 operands
with per-tensor scales on the block-scaled MFMA (cn_conv_fwd_fp8, 2x the bf16 MFMA rate);
everything else -- BatchNorm, activations, the co-attention, the whole backward (which reads
the bf16 activations saved by the forward), the fp32 master weights and SGD -- stays as in the
bf16 path.

* Weights: current scaling.  Each conv weight has an fp8 copy [Cout][KH*KW*Cin] and a scale
  state; after every SGD step all copies are re-quantised from the fp32 masters in three
  launches (cn_fp8_quant_multi: amax, scale, quantise), inside the recorded step graph.
* Activations: delayed scaling.  A conv input is quantised once per forward (shared by the
  convs that read it) with the scale derived from the previous step's amax of that tensor,
  while this step's amax is collected; one cn_fp8_update per encoder pass advances all scales.
  A state is calibrated (amax pass) on first use, so step 0 does not saturate.
* Gradients (dgrad): the output gradient of a compute-heavy stride-1 conv (K = kh*kw*Cout >=
  2304: the 3x3 layer-3/4 convs, the ASPP convs) is quantised to e5m2 (range over precision,
  the usual gradient format) with delayed scaling of its own (Fp8Context.grads, updated once
  per encoder backward), and multiplied with an e4m3 copy of the transposed weight (current
  scaling, refreshed with the forward copies after every SGD step) -- cn_conv_dgrad_fp8, the
  block-scaled MFMA with A format e5m2.
* Weight gradients of the same convs (round 5): the e5m2 output gradient above times the e4m3
  input copy the forward conv read (kept for the backward with the scale it was quantised with:
  Fp8Acts.end() snapshots the pass's scales before advancing them) -- cn_conv_wgrad_fp8, both
  operands k-major through ds_read_b64_tr_b8; the bottlenecks' 3x3 convs grouped per layer like
  the bf16 ones.  The 1x1 / shallow weight gradients (no e5m2 dY) stay bf16 x bf16.
"""
import struct
import weakref

import numpy as np
import torch

from . import _native as nv
from . import ops

_REC = struct.Struct("<QqiiQqQq")   # Fp8Rec (fp8.hip): x, ldx, P, C, y, ldy, state, x_is_bf16
assert _REC.size == 56


def fp8_ok(x, cin):
    return x.dtype == torch.bfloat16 and cin % 16 == 0 and ops.ld(x) % 16 == 0


class Fp8Weights:
    """fp8 copies of fp32 conv weights (channels_last), refreshed after each optimiser step."""

    def __init__(self):
        self._c = {}          # id(w) -> [wf8, state, tag, w, src]; ("t", id(w)) -> the transposed
                              # dgrad copy (src = the bf16 [Cin][KH*KW*Cout] weight-cache copy)
        self._table = None
        self._table_n = 0
        self._table_ptrs = None   # the master / copy addresses the table was packed with
        self._captured = False    # a recorded graph replays the current table
        self._graph_tables = []   # tables read by recorded graphs: kept for their lifetime

    @staticmethod
    def _tag(w):
        return (w._version, w.data_ptr())

    def get(self, w):
        e = self._c.get(id(w))
        if e is None:
            if self._captured:
                raise RuntimeError("new fp8 weight after a graph captured this context's "
                                   "refresh table (re-capture the step)")
            cout = w.shape[0]
            k = w.numel() // cout
            wf8 = torch.empty((cout, k), dtype=torch.uint8, device=w.device)
            e = [wf8, ops.fp8_state(w.device), None, w, None]
            self._c[id(w)] = e
            self._table = None
        if e[2] != self._tag(w):
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("fp8 weight copy is stale inside a graph capture")
            cin = w.shape[1]
            nv.call("cn_fp8_quant", nv.DT_F32, w.data_ptr(), cin, w.numel() // cin, cin,
                    e[0].data_ptr(), cin, e[1].data_ptr(), ops.FP8_CURRENT, nv.stream())
            e[2] = self._tag(w)
        return e[0], e[1]

    def get_t(self, w, wt):
        """e4m3 copy of the transposed weight wt (bf16 [Cin][KH*KW*Cout], the dgrad operand of
        the weight cache), refreshed from wt with current scaling; (wt8, state)."""
        key = ("t", id(w))
        e = self._c.get(key)
        if e is None:
            if self._captured:
                raise RuntimeError("new fp8 weight after a graph captured this context's "
                                   "refresh table (re-capture the step)")
            e = [torch.empty(tuple(wt.shape), dtype=torch.uint8, device=wt.device),
                 ops.fp8_state(wt.device), None, w, wt]
            self._c[key] = e
            self._table = None
        if e[2] != self._tag(w):
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("fp8 weight copy is stale inside a graph capture")
            ops.fp8_quant(wt, e[1], ops.FP8_CURRENT, out=e[0])
            e[2] = self._tag(w)
        return e[0], e[1]

    def _ptrs(self):
        return tuple((e[3].data_ptr(), e[0].data_ptr(), e[1].data_ptr(),
                      e[4].data_ptr() if e[4] is not None else 0) for e in self._c.values())

    def refresh_all(self):
        """Re-quantise every fp8 copy from its (just updated) master: 3 launches."""
        if not self._c:
            return
        capturing = torch.cuda.is_current_stream_capturing()
        ptrs = self._ptrs()
        if self._table is not None and ptrs != self._table_ptrs:
            # a master's storage was replaced (p.data = ..., re-materialisation): the packed
            # table would refresh from the old buffer
            if self._captured or capturing:
                raise RuntimeError("fp8 weight storage moved after its refresh table was "
                                   "recorded in a graph (re-capture the step)")
            self._table = None
        if self._table is None:
            if capturing:
                raise RuntimeError("fp8 weight table must be built before graph capture")
            blob = b""
            for wf8, st, _, w, src in self._c.values():
                if src is None:   # forward copy from the fp32 master [Cout][KH][KW][Cin]
                    cin = w.shape[1]
                    blob += _REC.pack(w.data_ptr(), cin, w.numel() // cin, cin, wf8.data_ptr(), cin,
                                      st.data_ptr(), 0)
                else:             # transposed dgrad copy from the bf16 weight-cache copy
                    p_, c_ = src.shape
                    blob += _REC.pack(src.data_ptr(), ops.ld(src), p_, c_, wf8.data_ptr(), c_,
                                      st.data_ptr(), 1)
            host = torch.from_numpy(np.frombuffer(blob, dtype=np.uint8).copy())
            dev = next(iter(self._c.values()))[0].device
            self._table = host.to(dev)
            self._table_n = len(self._c)
            self._table_ptrs = ptrs
        if capturing:
            self._captured = True
            if not any(t is self._table for t in self._graph_tables):
                self._graph_tables.append(self._table)   # one reference per distinct table
        nv.call("cn_fp8_quant_multi", self._table.data_ptr(), self._table_n, nv.stream())
        for e in self._c.values():
            e[2] = self._tag(e[3]) if e[3] is not None else None

    def mark_updated(self):
        """The masters changed in place (SGD): copies valid after refresh_all()."""
        for e in self._c.values():
            e[2] = self._tag(e[3])


class Fp8Acts:
    """Delayed-scaling states of the conv inputs (e4m3) or of the dgrad output gradients
    (fmt=e5m2), in one device buffer (one update launch)."""

    def __init__(self, cap=1024, fmt=ops.FP8_E4M3):
        self.cap = cap
        self.fmt = fmt
        self.states = None
        self.slots = {}
        self.calibrated = set()
        self.pass_cache = {}
        self.handle = None

    def slot_of(self, st):
        """Slot index of a state view returned by state() / quant()."""
        return (st.data_ptr() - self.states.data_ptr()) // (4 * self.states.element_size())

    def saved(self, x8, st):
        """(x8, pass handle, slot): what a backward needs to dequantise x8 after end() advanced
        the live scale -- the handle's snapshot holds the scale x8 was quantised with."""
        return (x8, self.handle, self.slot_of(st))

    def begin(self):
        self.pass_cache = {}
        self.handle = PassScales()

    def state(self, key, device):
        if self.states is None:
            self.states = torch.tensor([[1.0, 1.0, 0.0, ops.FMT_MAX[self.fmt]]] * self.cap,
                                       dtype=torch.float32, device=device)
        i = self.slots.get(key)
        if i is None:
            i = len(self.slots)
            if i >= self.cap:
                raise RuntimeError("too many fp8 activation states")
            self.slots[key] = i
        return i, self.states[i]

    def quant(self, x, key):
        """x8 of x (bf16 [P, C]) under this key's delayed scale; cached for the pass."""
        ck = (x.data_ptr(), tuple(x.shape), ops.ld(x))
        hit = self.pass_cache.get(ck)
        if hit is not None:
            return hit[0], hit[1]
        i, st = self.state(key, x.device)
        if i not in self.calibrated:   # first use: this tensor's own amax sets the scale
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("fp8 activation state first used inside a graph capture")
            ops.fp8_quant(x, st, ops.FP8_AMAX, fmt=self.fmt)
            ops.fp8_update(st)
            self.calibrated.add(i)
        x8 = ops.fp8_quant(x, st, ops.FP8_DELAYED, fmt=self.fmt)
        self.pass_cache[ck] = (x8, st, x)   # x held: its address cannot be reused this pass
        return x8, st

    def ready(self, key, device):
        """(slot state) if this key's scale is calibrated (a producer may quantise in its own
        pass), else None."""
        i, st = self.state(key, device)
        return st if i in self.calibrated else None

    def register(self, x, x8, st):
        """x8 / st are the fp8 copy of x produced elsewhere (bn_apply's fused output)."""
        self.pass_cache[(x.data_ptr(), tuple(x.shape), ops.ld(x))] = (x8, st, x)

    def end(self):
        """Advance every used scale from the amax collected in this pass (one launch).  The
        scales this pass quantised with are kept first (one copy into the pass handle): the fp8
        weight gradients of the backward read the e4m3 activation copies of this forward."""
        self.pass_cache = {}
        if self.slots:
            if self.handle is not None:
                self.handle.snap = self.states[:len(self.slots)].clone()
            ops.fp8_update(self.states[:len(self.slots)])


class PassScales:
    """The scale states of one forward pass as they were while it quantised (Fp8Acts.end())."""

    def __init__(self):
        self.snap = None

    def state(self, slot):
        if self.snap is None:
            raise RuntimeError("fp8 pass scales read before the pass ended")
        return self.snap[slot]


class Fp8Context:
    """One model's fp8 state: weight copies + activation scales (model.set_fp8 creates it; the
    modules reach it through their `_cn_fp8` attribute).  Per model, so that a state is never
    picked up by another model whose modules happen to reuse a freed object's id."""

    def __init__(self):
        self.weights = Fp8Weights()
        self.acts = Fp8Acts()
        self.grads = Fp8Acts(fmt=ops.FP8_E5M2)
        LIVE.add(self)


LIVE = weakref.WeakSet()


def contexts_of(params):
    """The live fp8 contexts holding a weight copy of any of `params` (an optimiser's own)."""
    ids = {id(p) for p in params}
    return [ctx for ctx in list(LIVE) if any(k in ids for k in ctx.weights._c)]


def refresh_weights_of(params):
    """After an optimiser step: re-quantise the fp8 copies of the contexts whose weights this
    optimiser trains -- never another model's (its table is not tied to this step's graph)."""
    for ctx in contexts_of(params):
        ctx.weights.refresh_all()
