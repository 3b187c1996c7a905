"""One training iteration of the reference loop, replayed as a HIP graph.

Reference loop body (train.py:560-602, --model raa):
    pred_a, pred_b, _ = model(rgb_a, rgb_b, depth_a, depth_b)
    loss = calc_loss_BCE(pred_a, gt_a) + 0.8 * calc_loss_L1(pred_a, gt_a)
         + calc_loss_BCE(pred_b, gt_b) + 0.8 * calc_loss_L1(pred_b, gt_b)
    optimizer.zero_grad(); loss.backward(); optimizer.step()
with the poly learning rate set before each step (train.py:171-172, :348-355).

The eager step issues ~2000 kernel launches from Python, so at this model size the host, not
the GPU, sets the pace.  TrainStep records the whole iteration once (forward of both frames x
both encoders, co-attention, decoder, loss, hand-written backward, SGD) into a HIP graph and
replays it: one host call per step.  Per-step inputs live in static device tensors (load()),
the learning rates in a device tensor refreshed before each replay, and the BCE positive
counts (the only data-dependent scalar of the step) are computed ahead of the graph — under
data parallelism they are all-reduced there, so the graph itself holds no collective.

Data parallel (world > 1): every gradient lives in one flat fp32 "arena" laid out in the order
the backward produces it, cut into buckets: [head (co-attention, fusion, decoder)] then the
depth encoder and the RGB encoder segment by segment ([ASPP + layer4], layer3 halves,
[layer2 + layer1 + stem]).  The encoder backwards are deferred out of autograd
(encoder_fn.DeferredEncoderBwd) and write their gradients straight into their bucket, so
nothing is packed.  The step is recorded as a chain of HIP graphs -- forward + autograd
backward of the head, then one graph per encoder segment, then SGD -- and each bucket's
all-reduce (RCCL, async, pre-scaled by 1/world and summed = DataParallel's mean) is issued on
the host as soon as its graph is queued: bucket k reduces over xGMI while segment k+1
computes.  Optionally the buckets are reduced in bf16 (grad_dtype="bf16": half the bytes).
BN running statistics stay per rank during training (train-mode BN normalises with batch
statistics, so they never enter the step); sync_buffers() broadcasts rank 0's before evaluation
or checkpointing.
"""
import os

import torch
import torch.distributed as dist

from . import _native as nv
from . import functions as fn
from . import ops


class TrainStep:
    """`size` = H (square frames) or (H, W); `batch` = frame pairs on this rank."""

    def __init__(self, model, opt, batch, size, l1_weight=0.8, graphed=True, group=None,
                 grad_dtype="fp32", split_graphs=None):
        self.model, self.opt = model, opt
        # split_graphs (single process, encoders on two streams): record the step as one-stream
        # graphs per phase and stream instead of one graph with a forked branch (_split_capture).
        # ROCm's launch of a multi-stream graph blocks the host for ~the replay's duration; the
        # one-stream graphs return at once (0.8 ms per step), so the host's own work between
        # steps (the loader's decode / augmentation in train.py) overlaps the device's step.  The
        # device time per step is the same either way (profiles/r04_split_graphs_ab.txt).
        if split_graphs is None:
            split_graphs = os.environ.get("CN_SPLIT_GRAPHS", "1") == "1"
        self.split_graphs = bool(split_graphs)
        self._split = None
        self.grad_dtype = grad_dtype
        self.l1 = float(l1_weight)
        self.graphed = graphed
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        dev = next(model.parameters()).device
        b = batch
        h, w = (size, size) if isinstance(size, int) else tuple(size)
        self.hw = (h, w)
        self.rgb_a = torch.zeros((b, 3, h, w), device=dev)
        self.rgb_b = torch.zeros_like(self.rgb_a)
        self.dep_a = torch.zeros((b, 1, h, w), device=dev)
        self.dep_b = torch.zeros_like(self.dep_a)
        self.gt_a = torch.zeros((b, 1, h, w), device=dev)
        self.gt_b = torch.zeros_like(self.gt_a)
        self.cnt = torch.zeros((2,), dtype=torch.int64, device=dev)
        self.total = b * h * w * self.world
        self.loss = torch.zeros((), dtype=torch.float32, device=dev)
        self._one = torch.ones((), dtype=torch.float32, device=dev)
        self.mem_hook = None   # callable(prefix): the reference's logMem (train.py:51-58)
        self._capturing = False
        # every eager iteration AND the capture run on this one stream: autograd pins each
        # parameter's AccumulateGrad node to the stream it was created on
        self.stream = torch.cuda.Stream(device=dev) if dev.type == "cuda" else None
        self.params = []
        seen = set()
        for g in opt.groups:
            for p in g:
                if id(p) not in seen:
                    seen.add(id(p))
                    self.params.append(p)
        self.flat = None
        self.graph = None
        self._nbt_delta = None
        self.dp = None            # data-parallel state (_dp_setup)
        opt.reserve()  # pinned SGD tables + the device learning-rate tensor

    # ---- inputs ---------------------------------------------------------------------------
    def load(self, rgb_a, rgb_b, dep_a, dep_b, gt_a, gt_b):
        for dst, src in zip((self.rgb_a, self.rgb_b, self.dep_a, self.dep_b, self.gt_a, self.gt_b),
                            (rgb_a, rgb_b, dep_a, dep_b, gt_a, gt_b)):
            dst.copy_(src, non_blocking=True)

    def _counts(self):
        """Global #(gt >= 0.5) of both frames (train.py:183-187), before the graph."""
        fn.count_positive(self.gt_a, out=self.cnt[0:1])
        fn.count_positive(self.gt_b, out=self.cnt[1:2])
        if self.world > 1:
            dist.all_reduce(self.cnt, group=self.group)

    def _mem(self, prefix):
        if self.mem_hook is not None and not self._capturing:
            self.mem_hook(prefix)

    def _on_stream(self, fn_, *a):
        """Run fn_ on self.stream (ordered after the caller's current stream and back)."""
        if self.stream is None:
            return fn_(*a)
        cur = torch.cuda.current_stream()
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            r = fn_(*a)
        cur.wait_stream(self.stream)
        return r

    # ---- the recorded body -------------------------------------------------------------------
    def _body(self):
        self.opt.zero_grad()
        x1, x2, _ = self.model(self.rgb_a, self.rgb_b, self.dep_a, self.dep_b)
        loss = fn.BceL1PairDevFn.apply(x1, x2, self.gt_a, self.gt_b, self.cnt, self.total, self.l1)
        self._mem(" After forward")
        # d loss / d loss = 1 from a preallocated device scalar (no fill kernel per step)
        torch.autograd.backward(loss, self._one)
        self._mem(" After backward")
        self.loss = loss.detach()
        self.opt.step()

    # ---- split recording: one-stream graphs per phase and stream -------------------------------
    def _split_ok(self):
        m = self.model
        return (self.split_graphs and self.world == 1 and self.stream is not None
                and getattr(m, "pair_encoder", False) and getattr(m, "no_grad_for_counterpart", False)
                and m._side_stream(self.rgb_a.device) is not None
                and self.rgb_a.shape == self.rgb_b.shape)

    def _split_capture(self, s1):
        """The step as six one-stream graphs, the model's forward / backward cut at its four
        cross-stream edges (rgbd_segmentation_RAA.forward: depth encoder + depth head on the side
        stream, joined before the decoder; autograd runs their backward there too):
            s1: A  RGB encoder + RGB head       s2: A' depth encoder + depth head
            s1: B  decoder + loss + their backward (gradients of the three head outputs)
            s1: C  RGB head + encoder backward  s2: C' depth head + encoder backward
            s1: D  SGD
        Each stream's graphs draw on a pool of their own: a graph of one stream never reuses
        memory a concurrently running graph of the other stream still holds.  The kernels and
        their order per stream are those of the one-graph recording (bitwise-equal results,
        tests/test_gpu_train_step.py)."""
        from .encoder_fn import encode_pair
        m = self.model
        s2 = m._side_stream(self.rgb_a.device)
        p1, p2 = torch.cuda.graph_pool_handle(), torch.cuda.graph_pool_handle()
        isz = tuple(self.rgb_a.shape[2:])
        self.opt.zero_grad()
        m._set_dtype()
        s2.wait_stream(s1)
        gA, hA, gB, gC, hC, gD = (torch.cuda.CUDAGraph() for _ in range(6))
        with torch.cuda.graph(gA, stream=s1, pool=p1):
            va, vb, geo = encode_pair(m.encoder, self.rgb_a, self.rgb_b)
            with torch.no_grad():
                m.encoder.annotate_nhwc(vb, geo, isz)                      # labels (:146)
            z_a, z_b = m._rgb_head(va, vb, geo)
        with torch.cuda.graph(hA, stream=s2, pool=p2):
            da, db, dgeo = encode_pair(m.depth_encoder, self.dep_a, self.dep_b)
            dz_a, dz_b = m._depth_head(da, db, dgeo)
        if dgeo != geo:
            raise RuntimeError("RGB and depth feature maps differ: %s vs %s" % (geo, dgeo))
        outs = [t for t in (z_a, z_b, dz_a) if t.requires_grad]
        dec = [p for mod in (m.segmentation_classifier_A, m.segmentation_classifier_B)
               for p in mod.parameters() if p.requires_grad]
        with torch.cuda.graph(gB, stream=s1, pool=p1):
            x1, x2 = m._decode(z_a, z_b, dz_a, dz_b, geo, isz)
            loss = fn.BceL1PairDevFn.apply(x1, x2, self.gt_a, self.gt_b, self.cnt, self.total, self.l1)
            grads = torch.autograd.grad(loss, outs + dec, self._one)
            for p, g in zip(dec, grads[len(outs):]):
                p.grad = g
        gout = dict(zip([id(t) for t in outs], grads[:len(outs)]))
        rgb = [(t, gout[id(t)]) for t in (z_a, z_b) if id(t) in gout]
        with torch.cuda.graph(gC, stream=s1, pool=p1):
            torch.autograd.backward([t for t, _ in rgb], [g for _, g in rgb])
        with torch.cuda.graph(hC, stream=s2, pool=p2):
            if id(dz_a) in gout:
                torch.autograd.backward([dz_a], [gout[id(dz_a)]])
        with torch.cuda.graph(gD, stream=s1, pool=p1):
            self.opt.step()
        self.loss = loss.detach()
        # the graphs read these across their boundaries: keep them (and their memory) alive
        self._split = {"s2": s2, "g": (gA, hA, gB, gC, hC, gD),
                       "keep": (va, vb, z_a, z_b, da, db, dz_a, dz_b, x1, x2, grads)}
        self.graph = gA

    def _split_replay(self):
        sp = self._split
        s2 = sp["s2"]
        gA, hA, gB, gC, hC, gD = sp["g"]
        cur = torch.cuda.current_stream()
        s2.wait_stream(cur)              # inputs, counts and learning rates of this step
        with torch.cuda.stream(s2):
            hA.replay()
        gA.replay()
        cur.wait_stream(s2)
        gB.replay()
        s2.wait_stream(cur)
        with torch.cuda.stream(s2):
            hC.replay()
        gC.replay()
        cur.wait_stream(s2)
        gD.replay()

    # ---- data parallel: arena, buckets, deferred encoder backward ----------------------------
    def _bind(self):
        """Point the encoders' deferred-backward holders at THIS step's (several TrainSteps may
        share one model: ShapeGraphCache keeps one per frame size)."""
        if self.dp is not None:
            for e, d in zip((self.model.encoder, self.model.depth_encoder), self.dp["defers"]):
                e._cn_defer = d

    def _dp_setup(self):
        from .encoder_fn import DeferredEncoderBwd
        m = self.model
        train = [p for p in self.params]
        encs = [m.encoder, m.depth_encoder]
        defers = [DeferredEncoderBwd(e, None) for e in encs]
        enc_ids = {id(p) for e in encs for p in e.parameters()}
        head = [p for p in train if id(p) not in enc_ids]
        buckets = [head]
        # stage j = RGB segment j (on the step's stream) beside depth segment j (on the model's
        # second stream, as in the forward); one bucket per stage, all-reduced while the next
        # stage computes
        segs = []
        for j in range(max(len(d.plan) for d in defers)):
            st = [(d, j) for d in defers if j < len(d.plan)]
            ps = [p for d, k in st for p in d.segment_params(k) if any(p is q for q in train)]
            buckets.append(ps)
            segs.append(st)
        got = [p for b in buckets for p in b]
        assert len({id(p) for p in got}) == len(got), "a parameter in two buckets"
        missing = [p for p in train if id(p) not in {id(q) for q in got}]
        buckets[0] += missing   # trainable encoder params outside the plan (none in RAA)
        # every slot starts on a 64-byte boundary (the per-channel kernels need 16-B alignment)
        rnd = lambda k: (k + 15) // 16 * 16
        n = sum(rnd(p.numel()) for b in buckets for p in b)
        dev = train[0].device
        flat = torch.zeros((n,), dtype=torch.float32, device=dev)
        arena, views, ranges, off = {}, {}, [], 0
        for b in buckets:
            b0 = off
            for p in b:
                sl = flat[off:off + p.numel()]
                arena[p] = sl
                views[p] = sl.as_strided(p.shape, p.stride())
                off += rnd(p.numel())
            ranges.append((b0, off))
        for d in defers:
            d.arena = arena
        for e, d in zip(encs, defers):
            e._cn_defer = d
        half = None
        if self.grad_dtype == "bf16":
            half = torch.zeros((n,), dtype=torch.bfloat16, device=dev)
        self.dp = {"buckets": buckets, "ranges": ranges, "segs": segs, "flat": flat, "arena": arena,
                   "views": views, "head": head, "half": half, "works": [], "graphs": None,
                   "head_live": None, "defers": defers}
        self.flat = flat

    def _dp_forward_backward(self):
        """Graph A's body: forward, loss, autograd backward (encoders deferred), head bucket."""
        dp = self.dp
        self.opt.zero_grad()
        x1, x2, _ = self.model(self.rgb_a, self.rgb_b, self.dep_a, self.dep_b)
        loss = fn.BceL1PairDevFn.apply(x1, x2, self.gt_a, self.gt_b, self.cnt, self.total, self.l1)
        self._mem(" After forward")
        torch.autograd.backward(loss, self._one)
        self.loss = loss.detach()
        if dp["head_live"] is None:   # which head parameters receive a gradient (static)
            dp["head_live"] = [p for p in dp["head"] if p.grad is not None]
        live = dp["head_live"]
        torch._foreach_copy_([dp["views"][p] for p in live], [p.grad for p in live])
        self._dp_prepare_bucket(0)

    def _dp_prepare_bucket(self, k):
        """Device work that readies bucket k for its all-reduce: the 1/world pre-scale (sum of
        scaled = DataParallel's mean) and, for bf16 reduction, the cast."""
        dp = self.dp
        a, b = dp["ranges"][k]
        if b == a:
            return
        nv.call("cn_scale", dp["flat"][a:].data_ptr(), b - a, 1.0 / self.world, nv.stream())
        if dp["half"] is not None:
            ops.cast_copy(dp["flat"][a:b].view(-1, 1), dp["half"][a:b].view(-1, 1))

    def _dp_stage(self, i):
        """Encoder-backward stage i: the RGB segment here, the depth segment on the side stream."""
        st = self.dp["segs"][i]
        # the stream follows the ENCODER, not the position in the stage: the depth segments'
        # saved activations were allocated on the side stream by the forward
        depth = getattr(self.model.depth_encoder, "_cn_defer", None)
        on_side = [(d, k) for d, k in st if d is depth]
        here = [(d, k) for d, k in st if d is not depth]
        side = self.model._side_stream(self.flat.device) if on_side else None
        if side is None:
            for d, k in st:
                d.run(k)
            return
        cur = torch.cuda.current_stream()
        side.wait_stream(cur)
        for d, k in here:
            d.run(k)
        with torch.cuda.stream(side):
            for d, k in on_side:
                d.run(k)
        cur.wait_stream(side)

    def _dp_segment(self, i):
        self._dp_stage(i)
        self._dp_prepare_bucket(i + 1)

    def _dp_launch_reduce(self, k):
        """Issue bucket k's all-reduce (async): RCCL waits for the work queued so far on the
        current stream and runs beside the segments queued after it."""
        dp = self.dp
        a, b = dp["ranges"][k]
        if b == a:
            return
        buf = dp["half"][a:b] if dp["half"] is not None else dp["flat"][a:b]
        dp["works"].append(dist.all_reduce(buf, group=self.group, async_op=True))

    def _dp_finish(self):
        """Wait for every bucket, (cast back,) point the parameters' .grad at the arena, SGD."""
        dp = self.dp
        for w in dp["works"]:
            w.wait()
        dp["works"] = []
        self._dp_sgd()

    def _dp_sgd(self):
        dp = self.dp
        if dp["half"] is not None:
            ops.cast_copy(dp["half"].view(-1, 1), dp["flat"].view(-1, 1))
        live = set(id(p) for p in dp["head_live"])
        for b_i, b in enumerate(dp["buckets"]):
            for p in b:
                if b_i > 0 or id(p) in live:
                    p.grad = dp["views"][p]
        self.opt.step()
        self._mem(" After backward")

    def _dp_eager_once(self):
        self._dp_forward_backward()
        self._dp_launch_reduce(0)
        for i in range(len(self.dp["segs"])):
            self._dp_segment(i)
            self._dp_launch_reduce(i + 1)
        self._dp_finish()

    # ---- capture / replay ---------------------------------------------------------------------
    def _bn_counts(self):
        return {m: getattr(m, "_cn_nbt", 0) for m in self.model.modules()
                if isinstance(m, torch.nn.modules.batchnorm._BatchNorm)}

    def capture(self, warmup=2):
        """Run `warmup` eager iterations (they are real steps) on a side stream, then record."""
        if self.world > 1 and self.dp is None:
            self._dp_setup()
        self._bind()
        if not self.graphed:
            for _ in range(warmup):
                self._eager_once()
            return
        # warm up AND record on one side stream (self.stream): autograd pins each parameter's
        # gradient accumulator to the stream it was created on, and an accumulation (a
        # parameter used twice) running on any other stream than the capturing one would
        # escape the graph
        s = self.stream
        for _ in range(warmup):
            self._eager_once()
        warm_loss = self.loss.clone() if warmup else None   # the last real step's loss
        torch.cuda.synchronize()
        self.opt.reserve()
        self.opt.freeze_for_capture()
        self.opt.refresh_lrs()
        torch.cuda.synchronize()
        before = self._bn_counts()
        self._capturing = True
        try:
            if self.world > 1:
                self._dp_capture(s)
            elif self._split_ok():
                self._split_capture(s)
            else:
                self.graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(self.graph, stream=s):
                    self._body()
        finally:
            self._capturing = False
        self._graph_loss = self.loss
        if warm_loss is not None:
            self.loss = warm_loss   # recording computed nothing: report the warm-up step's loss
        after = self._bn_counts()
        self._nbt_delta = {m: after[m] - before[m] for m in after if after[m] != before[m]}
        for m, k in before.items():  # recording executed nothing: only replays count
            m._cn_nbt = k
        torch.cuda.synchronize()

    def _dp_capture(self, s):
        """Record the data-parallel step as a chain of graphs sharing one memory pool: A (forward
        + autograd backward + head bucket), one per encoder segment, and SGD.  The tensors the
        later graphs read (saved activations, the stashed feature gradients) stay referenced
        by the deferred-backward holders, so no capture reuses their memory."""
        dp = self.dp
        pool = torch.cuda.graph_pool_handle()
        keep = []
        ga = torch.cuda.CUDAGraph()
        with torch.cuda.graph(ga, stream=s, pool=pool):
            self._dp_forward_backward()
        segs = []
        for i in range(len(dp["segs"])):
            keep.append([(d.rec, d.dfa) for d, _ in dp["segs"][i]])
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s, pool=pool):
                self._dp_segment(i)
            segs.append(g)
        gs = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gs, stream=s, pool=pool):
            self._dp_sgd()
        dp["graphs"] = (ga, segs, gs, keep)
        self.graph = ga

    def _dp_replay(self):
        dp = self.dp
        ga, segs, gs, _ = dp["graphs"]
        ga.replay()
        self._dp_launch_reduce(0)
        for i, g in enumerate(segs):
            g.replay()
            self._dp_launch_reduce(i + 1)
        for w in dp["works"]:
            w.wait()
        dp["works"] = []
        gs.replay()

    def run_batch(self, rgb_a, rgb_b, dep_a, dep_b, gt_a, gt_b, lrs):
        """One EAGER iteration on inputs of any size (the reference's augmented batches change
        H, W every batch, so they cannot replay one recorded graph)."""
        if self.graphed and self.graph is not None:
            raise RuntimeError("run_batch is the eager path; build the TrainStep with graphed=False")
        if self.world > 1 and self.dp is None:
            self._dp_setup()
        b, _, h, w = rgb_a.shape
        self.rgb_a, self.rgb_b, self.dep_a, self.dep_b, self.gt_a, self.gt_b = (
            rgb_a, rgb_b, dep_a, dep_b, gt_a, gt_b)
        self.hw = (h, w)
        self.total = b * h * w * self.world
        self.opt.set_lrs(lrs)
        self._eager_once()
        return self.loss

    def eager(self, lrs):
        """One eager (un-graphed) iteration, e.g. to time its kernels with HIP events."""
        self.opt.set_lrs(lrs)
        self._eager_once()
        return self.loss

    def _eager_once(self):
        if self.world > 1 and self.dp is None:
            self._dp_setup()
        self._bind()

        def once():
            self._counts()
            self.opt.refresh_lrs()
            if self.world > 1:
                self._dp_eager_once()
            else:
                self._body()
        self._on_stream(once)

    def __call__(self, lrs):
        """One iteration on the loaded inputs with learning rates `lrs` (one per group)."""
        self.opt.set_lrs(lrs)
        if self.graph is None:
            self._eager_once()
            return self.loss
        self.opt.refresh_lrs()
        self._counts()
        if self.world > 1:
            self._dp_replay()
        elif self._split is not None:
            self._split_replay()
        else:
            self.graph.replay()
        self.loss = self._graph_loss
        self._mem(" After forward")
        self._mem(" After backward")
        # the replay updated the fp32 masters AND their compute-dtype copies in place (cn_sgd):
        # the weight cache stays valid
        for m, d in self._nbt_delta.items():
            m._cn_nbt = getattr(m, "_cn_nbt", 0) + d
        return self.loss

    def sync_buffers(self, src=0):
        """Broadcast rank `src`'s BN running statistics (before eval / checkpoint)."""
        if self.world > 1:
            for b in self.model.buffers():
                dist.broadcast(b, src, group=self.group)


class ShapeGraphCache:
    """Recorded steps keyed by frame size, for inputs whose size changes from batch to batch (the
    SBM-RGBD loader's per-batch random scale x crop, dataloaders/sbm_rgbd_loader.py:700-702,
    :710-722): a size seen `min_hits` times gets its own TrainStep, recorded on that batch (the
    recording run is a real eager step) and replayed on every later batch of that size; other
    sizes run eagerly (TrainStep.run_batch).  Up to `capacity` sizes are kept (least recently used
    evicted: its graph and memory pool are released).  All steps share the model, the optimiser
    and its state, so the trajectory is the same whichever path a batch takes (graph replay and
    eager step run the same kernels in the same order: bitwise equal)."""

    def __init__(self, model, opt, batch, l1_weight=0.8, grad_dtype="fp32", capacity=24, min_hits=2):
        from collections import OrderedDict
        self.model, self.opt, self.batch = model, opt, batch
        self.l1, self.grad_dtype = l1_weight, grad_dtype
        self.capacity, self.min_hits = capacity, min_hits
        self.graphs = OrderedDict()      # (h, w) -> TrainStep (recorded)
        self.seen = {}
        self.evicted = set()             # sizes whose graph was evicted: never recorded again
        self.eager = None
        self.hits = self.records = self.eager_steps = 0

    def admit(self, hw, batch):
        """Policy for a batch of frame size `hw`: "hit" (replay its graph), "record" (record a
        graph for it now; the LRU graph is evicted when full) or "eager".  A size is recorded
        on its `min_hits`-th occurrence and at most once: an evicted size stays eager, so a
        stream of non-recurring sizes cannot make every batch pay a capture (each costs an
        eager step, a capture, an instantiation and a private memory pool)."""
        if hw in self.graphs:
            self.graphs.move_to_end(hw)
            self.hits += 1
            return "hit"
        self.seen[hw] = self.seen.get(hw, 0) + 1
        if (self.seen[hw] >= self.min_hits and self.capacity > 0 and batch == self.batch
                and hw not in self.evicted):
            if len(self.graphs) >= self.capacity:
                old, _ = self.graphs.popitem(last=False)
                self.evicted.add(old)
            self.graphs[hw] = None
            self.records += 1
            return "record"
        self.eager_steps += 1
        return "eager"

    def __call__(self, rgb_a, rgb_b, dep_a, dep_b, gt_a, gt_b, lrs):
        hw = tuple(rgb_a.shape[2:])
        ins = (rgb_a, rgb_b, dep_a, dep_b, gt_a, gt_b)
        act = self.admit(hw, rgb_a.shape[0])
        if act == "hit":
            st = self.graphs[hw]
            st.load(*ins)
            return st(lrs)
        if act == "record":
            st = TrainStep(self.model, self.opt, self.batch, hw, l1_weight=self.l1, graphed=True,
                           grad_dtype=self.grad_dtype)
            st.load(*ins)
            self.opt.set_lrs(lrs)
            try:
                st.capture(warmup=1)      # this batch's step runs eagerly, then the record
            except BaseException:
                # admit() reserved the slot: a failed recording (OOM, capture error) must not
                # leave a placeholder that the next batch of this size would "hit"
                self.graphs.pop(hw, None)
                self.evicted.add(hw)
                raise
            self.graphs[hw] = st
            return st.loss
        if self.eager is None:
            self.eager = TrainStep(self.model, self.opt, self.batch, hw, l1_weight=self.l1,
                                   graphed=False, grad_dtype=self.grad_dtype)
        return self.eager.run_batch(*ins, lrs)

    def sync_buffers(self, src=0):
        st = self.eager or next(iter(self.graphs.values()), None)
        if st is not None:
            st.sync_buffers(src)
