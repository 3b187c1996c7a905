"""SGD with momentum + weight decay as one multi-tensor HIP launch (cn_sgd), with the
reference's two parameter groups and poly learning-rate schedule.

Reference: optim.SGD([{get_1x_lr_params}, {get_10x_lr_params}], lr, momentum=0.9,
weight_decay=5e-4) (train.py:538-540), adjust_learning_rate / lr_poly (train.py:161-174,
:348-355), optimizer.step() (train.py:602).  Update rule = torch.optim.SGD (dampening 0,
no nesterov): d = g + wd*p ; buf = d on the first step, else momentum*buf + d ; p -= lr*buf.

`duplicate_params=True` reproduces the reference's quirk that get_1x_lr_params yields every
RGB-encoder parameter once per enclosing module: the update is applied
once per occurrence, in order (torch's for-loop SGD semantics).
"""
import struct

import numpy as np
import torch

from . import _native as nv
from .ops import WCACHE, WeightCache

# SgdTensor (ew.hip): p, g, buf, n, group, first, wf, wt, cout, khw, cin, cp, wdt, mode, beg, end
_REC = struct.Struct("<QQQqiiQQiiiiiiqq")
_FLAT_CHUNK = 1 << 16      # elements per flat work item
_TILE_CHUNK = 16           # 64x64 tiles per tiled work item


def reference_param_groups(model, duplicate_params=False):
    """(group0, group1) parameter lists as train.py:220-303 builds them for --model raa."""
    g0 = []
    for mod in model.get_params("encoder"):
        for sub in mod.modules():
            for p in sub.parameters():
                if p.requires_grad:
                    g0.append(p)
    if not duplicate_params:
        seen = set()
        g0 = [p for p in g0 if not (id(p) in seen or seen.add(id(p)))]
    g1 = []
    for sub in ("rgb_attention", "depth", "decoder"):
        for mod in model.get_params(sub):
            g1.extend(mod.parameters())
    return g0, g1


def lr_poly(base_lr, it, max_iter, power, epoch):
    """train.py:348-355"""
    factor = 1 if epoch < 6 else 0.5
    return base_lr * factor * ((1 - float(it) / max_iter) ** power)


class SGD:
    def __init__(self, groups, lrs, momentum=0.9, weight_decay=5e-4):
        self.groups = [list(g) for g in groups]
        self.lrs = list(lrs)
        self.momentum = float(momentum)
        self.weight_decay = float(weight_decay)
        self.state = {}
        self._tables = []
        self._table_key = None
        self._lr_dev = None
        self._lr_static = False
        self._stage = []      # [(pinned host uint8, device uint8)] per table
        self._stage_cap = []  # records each can hold
        self._graph_stage = []  # staging owned by recorded graphs (kept alive, never reused)

    def reserve(self, counts=None):
        """Allocate the pinned / device staging of the SGD tables (records per launch)."""
        if counts is None:
            counts = self._max_counts()
        dev = self.groups[0][0].device if self.groups[0] else self.groups[1][0].device
        self._stage, self._stage_cap = [], []
        for n in counts:
            host = torch.empty((max(n, 1) * _REC.size,), dtype=torch.uint8).pin_memory()
            self._stage.append((host, torch.empty_like(host, device=dev)))
            self._stage_cap.append(max(n, 1))
        self._table_key = None
        if self._lr_dev is None:
            self._lr_dev = torch.zeros((len(self.lrs),), dtype=torch.float32, device=dev)

    def _max_counts(self):
        """Upper bound of the work items per launch (step() splits launches at duplicates)."""
        counts, cur, seen = [], 0, set()
        for g in self.groups:
            for p in g:
                if id(p) in seen:
                    counts.append(cur)
                    cur, seen = 0, set()
                seen.add(id(p))
                n = p.numel()
                flat = -(-n // _FLAT_CHUNK)
                tiles = 0
                if p.dim() >= 2:
                    khw = p.shape[2] * p.shape[3] if p.dim() == 4 else 1
                    tiles = -(-(khw * (-(-p.shape[0] // 64)) * (-(-p.shape[1] // 64))) // _TILE_CHUNK)
                cur += max(1, flat, tiles)
        counts.append(cur)
        return counts

    def zero_grad(self, set_to_none=True):
        for g in self.groups:
            for p in g:
                if p.grad is not None:
                    if set_to_none:
                        p.grad = None
                    else:
                        p.grad.zero_()

    def set_lrs(self, lrs):
        self.lrs = list(lrs)

    def _records(self):
        """Work items of this step: (param record..., chunking) tuples for cn_sgd, plus the
        weight-cache entries the kernel refreshes."""
        recs, keep, refreshed = [], [], []
        start = {}
        for gi, g in enumerate(self.groups):
            for p in g:
                if p.grad is None:
                    continue
                if p.grad.dtype != torch.float32 or not _dense(p.grad, p):
                    p.grad = p.grad.contiguous(memory_format=_fmt(p))
                st = self.state.get(id(p))
                if st is None:
                    st = {"momentum_buffer": torch.empty_like(p), "steps": 0}
                    self.state[id(p)] = st
                # torch's for-loop SGD gathers every entry's momentum buffer BEFORE updating:
                # on a parameter's first step, each duplicate entry starts its own buffer
                # (buf = d), later steps share the one buffer
                if id(p) not in start:
                    start[id(p)] = st["steps"]
                first = int(start[id(p)] == 0)
                st["steps"] += 1
                buf = st["momentum_buffer"]
                ents = WCACHE.entries(p)
                copy = (0, 0, 0, 0, 0, 0, 0)
                if ents:
                    wf, wt, cout, khw, cin, cp, ent = ents[0]
                    wdt = 1 if wf.dtype == torch.bfloat16 else 2
                    copy = (wf.data_ptr(), wt.data_ptr() if wt is not None else 0, cout, khw, cin, cp, wdt)
                    refreshed.append(ent)
                    for e in ents[1:]:
                        WeightCache.invalidate(e[6])
                head = (p.data_ptr(), p.grad.data_ptr(), buf.data_ptr(), p.numel(), gi, first) + copy
                n = p.numel()
                cout, khw, cin = copy[2], copy[3], copy[4]
                if copy[6] and cin % 4 == 0 and n == cout * khw * cin:
                    ntiles = khw * (-(-cout // 64)) * (-(-cin // 64))
                    for b in range(0, ntiles, _TILE_CHUNK):
                        recs.append(head + (1, b, min(ntiles, b + _TILE_CHUNK)))
                else:
                    for b in range(0, n, _FLAT_CHUNK):
                        recs.append(head + (0, b, min(n, b + _FLAT_CHUNK)))
                keep.append(p)
        return recs, keep, refreshed

    @torch.no_grad()
    def step(self):
        recs, _, refreshed = self._records()
        if not recs:
            return
        dev = self.groups[0][0].device if self.groups[0] else self.groups[1][0].device
        # one launch per "generation" so a parameter listed k times is updated k times in
        # order (torch's for-loop SGD over duplicated param-group entries)
        batches, cur, seen = [], [], set()
        for r in recs:
            if (r[0], r[-2]) in seen:  # same parameter AND same work item: a duplicate entry
                batches.append(cur)
                cur, seen = [], set()
            cur.append(r)
            seen.add((r[0], r[-2]))
        batches.append(cur)
        self._upload_lrs(dev)
        key = tuple(tuple(b) for b in batches)
        if key != self._table_key:
            # device tables of SgdTensor records, staged through pinned memory so the copy is
            # asynchronous and capturable; rebuilt only when a pointer / flag changes.  The
            # pinned staging buffers are allocated once (reserve()) and rewritten in place, so
            # a rebuild inside a HIP-graph capture allocates nothing on the host.
            capturing = torch.cuda.is_current_stream_capturing()
            if not capturing and self._tables:
                torch.cuda.current_stream().synchronize()  # earlier copies out of the staging
            need = [len(b) for b in batches]
            if len(self._stage) < len(need) or any(c < n for c, n in zip(self._stage_cap, need)):
                if capturing:
                    raise RuntimeError("SGD.reserve() must size the tables before graph capture")
                self.reserve(need)
            self._tables = []
            for i, b in enumerate(batches):
                blob = b"".join(_REC.pack(*r) for r in b)
                host, devt = self._stage[i]
                host[:len(blob)].numpy()[:] = np.frombuffer(blob, dtype=np.uint8)
                devt[:len(blob)].copy_(host[:len(blob)], non_blocking=True)
                self._tables.append((host, devt, len(b)))
            self._table_key = key
            if capturing:
                # the recorded copy reads this staging at every replay: hand it to the graph
                # and never rewrite it (a later eager rebuild reserves a fresh set)
                self._graph_stage.append(self._stage)
                self._stage, self._stage_cap = [], []
        for host, devt, nrec in self._tables:
            nv.call("cn_sgd", devt.data_ptr(), nrec, self._lr_dev.data_ptr(), self.weight_decay,
                    self.momentum, nv.stream())
        # the kernel rewrote the compute-dtype copies of every updated parameter that has
        # one: those cache entries stay valid (no re-preparation before the next forward)
        for ent in refreshed:
            WCACHE.refreshed(ent)
        # fp8 copies (configs[4]): re-quantised from the new masters, 3 launches for all
        from .fp8 import refresh_weights_of
        refresh_weights_of(p for g in self.groups for p in g)

    def _upload_lrs(self, dev):
        if self._lr_dev is None:
            self._lr_dev = torch.empty((len(self.lrs),), dtype=torch.float32, device=dev)
        if self._lr_static:
            return  # refreshed outside a captured graph by refresh_lrs()
        self.refresh_lrs()

    def refresh_lrs(self):
        """Copy the current learning rates into the device tensor the SGD kernel reads.  A fresh
        pinned buffer per call: torch's caching host allocator keeps it until the copy ran."""
        host = torch.tensor(self.lrs, dtype=torch.float32).pin_memory()
        self._lr_dev.copy_(host, non_blocking=True)

    def freeze_for_capture(self):
        """After this, step() no longer re-uploads learning rates (use refresh_lrs())."""
        self._lr_static = True


def _fmt(p):
    if p.dim() == 4 and p.is_contiguous(memory_format=torch.channels_last):
        return torch.channels_last
    return torch.contiguous_format


def _dense(g, p):
    return g.is_contiguous(memory_format=_fmt(p)) and g.stride() == p.stride()
