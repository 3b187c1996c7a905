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

The step is recorded as a program of ONE-STREAM graphs cut at its cross-stream edges (the depth
side runs on a second stream): a graph with a forked branch blocks the host for its whole replay
on this ROCm, one-stream graphs joined by events outside the graphs do not (_program).

Data parallel (world > 1): every gradient lives in one flat fp32 "arena", cut into buckets:
[RGB head + decoder], [depth head], then each encoder segment by segment ([ASPP + layer4],
layer3 (halves for the RGB encoder), [layer2 + layer1 + stem]).  The encoder backwards are
deferred out of autograd (encoder_fn.DeferredEncoderBwd) and write their gradients straight
into their bucket, so nothing is packed.  Each segment is one graph on its encoder's stream, and
its bucket's all-reduce (RCCL, async, ReduceOp.AVG = DataParallel's mean; gloo: pre-scaled by
1/world and summed) is
issued on the host as soon as that graph is queued: bucket k reduces over xGMI while the later
segments compute.  Optionally the buckets are reduced in bf16 (grad_dtype="bf16": half the
bytes).  dp_chain=True runs the same chain at world 1 without collectives (timing / tracing);
collectives=True keeps the collectives at world 1 on an initialised process group (a world-1 RCCL
communicator is legal on one device: configs[2]'s per-rank step with RCCL really in the chain).
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

# Stream capture checks only the recording thread: with an nccl (RCCL) process group, its
# watchdog thread polls the events of finished all-reduces at any time, and under the default
# "global" mode one such poll landing inside a recording aborts the process (seen under rocprofv3,
# whose slower start moved the poll into the capture window).  Nothing else runs in other threads.
CAPTURE_MODE = "thread_local"


class TrainStep:
    """`size` = H (square frames) or (H, W); `batch` = frame pairs on this rank."""

    def __init__(self, model, opt, batch, size, l1_weight=0.8, graphed=True, group=None,
                 grad_dtype="fp32", split_graphs=None, dp_chain=None, collectives=None):
        self.model, self.opt = model, opt
        # split_graphs (encoders on two streams): record the step as one-stream graphs per phase
        # and stream (_program) instead of one graph with a forked branch.  ROCm's launch of a
        # multi-stream graph blocks the host for ~the replay's duration; the one-stream graphs
        # return at once (0.8 ms per step), so the host's own work between steps (train.py's
        # loader; its loss line is read one step late) overlaps the device's step.  The device
        # time per step is the same either way (profiles/r04_split_graphs_ab.txt).
        if split_graphs is None:
            split_graphs = os.environ.get("CN_SPLIT_GRAPHS", "1") == "1"
        self.split_graphs = bool(split_graphs)
        self.grad_dtype = grad_dtype
        self.l1 = float(l1_weight)
        self.graphed = graphed
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        # dp_chain: the data-parallel chain (gradient arena, staged encoder backward, per-bucket
        # pre-scale) at world 1, without collectives -- configs[2]'s per-rank step, timed and
        # traced on one GPU (bench.py --dp-chain 1).  CN_DP_CHAIN=1 sets it.
        if dp_chain is None:
            dp_chain = os.environ.get("CN_DP_CHAIN", "0") == "1"
        # collectives: issue the positive-count and bucket all-reduces even at world 1 (needs an
        # initialised process group, e.g. a world-1 "nccl" group = RCCL on this one device);
        # CN_DP_COLLECTIVES=1 sets it.  At world > 1 they are always issued.
        if collectives is None:
            collectives = os.environ.get("CN_DP_COLLECTIVES", "0") == "1"
        dist_on = dist.is_available() and dist.is_initialized()
        if collectives and not dist_on:
            raise RuntimeError("collectives=True needs an initialised torch.distributed process group")
        self.coll = self.world > 1 or (bool(collectives) and dist_on)
        self.dp_mode = self.world > 1 or bool(dp_chain) or self.coll
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
        self.graph = None         # first recorded graph (None: not recorded)
        self._rec = None          # recorded program: [("graph", role, g) | host actions]
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
        if self.coll:
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

    # ---- the one-piece body (eager single-process step, or one graph when not split) ---------
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

    # ---- the step as a program of one-stream pieces ------------------------------------------
    def _side(self):
        """The depth side's stream (None: the model runs its encoders on one stream)."""
        m = self.model
        if self.stream is None or not (getattr(m, "pair_encoder", False)
                                       and getattr(m, "no_grad_for_counterpart", False)
                                       and self.rgb_a.shape == self.rgb_b.shape):
            return None
        return m._side_stream(self.rgb_a.device)

    def _split_ok(self):
        return self.split_graphs and self.world == 1 and not self.dp_mode and self._side() is not None

    def _program(self):
        """The step cut at its cross-stream edges into one-stream pieces, in issue order:
            ("run", role, fn)         -- device work on stream `role` ("s1": the step's stream,
                                         "s2": the depth side's); ONE graph when recorded
            ("join", dst, src)        -- dst waits for src's queued work (outside the graphs)
            ("reduce", k, role)       -- bucket k's async all-reduce, issued from `role`
            ("finish",)               -- the step's stream waits for every issued all-reduce
        Forward: depth side (s2) | RGB side (s1) -- the model's rgb_side / depth_side, the same
        cut points as its forward(); then decoder + loss + their gradients (s1); the backward of
        each side on its own stream; SGD (s1).  Data parallel: each side's head backward ends with
        its head bucket and only stashes the encoder's feature gradient (DeferredEncoderBwd); the
        encoder backwards then run segment by segment (one piece each, RGB on s1 beside depth on
        s2), every piece ending with its bucket's pre-scale, and the host issues that bucket's
        all-reduce right after queuing it, so it runs over xGMI beside the later segments."""
        m = self.model
        dp = self.dp_mode
        env = {}
        isz = tuple(self.rgb_a.shape[2:])

        def dep_fwd():
            env["d"] = m.depth_side(self.dep_a, self.dep_b)

        def rgb_fwd():
            env["r"] = m.rgb_side(self.rgb_a, self.rgb_b, isz)

        def decode():
            va, vb, geo, labels, z_a, z_b = env["r"]
            da, db, dgeo, dz_a, dz_b = env["d"]
            x1, x2 = m.decode_outputs(z_a, z_b, dz_a, dz_b, geo, dgeo, isz)
            loss = fn.BceL1PairDevFn.apply(x1, x2, self.gt_a, self.gt_b, self.cnt, self.total, self.l1)
            self._mem(" After forward")
            outs = [t for t in (z_a, z_b, dz_a) if t.requires_grad]
            dec = [p for mod in (m.segmentation_classifier_A, m.segmentation_classifier_B)
                   for p in mod.parameters() if p.requires_grad]
            grads = torch.autograd.grad(loss, outs + dec, self._one)
            for p, g in zip(dec, grads[len(outs):]):
                p.grad = g
            env["gout"] = dict(zip([id(t) for t in outs], grads[:len(outs)]))
            env["loss"] = loss.detach()
            env["x"] = (x1, x2)

        def rgb_bwd():
            z_a, z_b = env["r"][4], env["r"][5]
            rgb = [(t, env["gout"][id(t)]) for t in (z_a, z_b) if id(t) in env["gout"]]
            torch.autograd.backward([t for t, _ in rgb], [g for _, g in rgb])
            if dp:
                self._dp_head_bucket(0)

        def dep_bwd():
            dz_a = env["d"][3]
            if id(dz_a) in env["gout"]:
                torch.autograd.backward([dz_a], [env["gout"][id(dz_a)]])
            if dp:
                self._dp_head_bucket(1)

        def sgd():
            if dp:
                self._dp_sgd()
            else:
                self.opt.step()
            self._mem(" After backward")

        prog = [("join", "s2", "s1"), ("run", "s2", dep_fwd), ("run", "s1", rgb_fwd),
                ("join", "s1", "s2"), ("run", "s1", decode), ("join", "s2", "s1"),
                ("run", "s2", dep_bwd)]
        if dp:
            prog.append(("reduce", 1, "s2"))
        prog.append(("run", "s1", rgb_bwd))
        if dp:
            prog.append(("reduce", 0, "s1"))
            for d, k, bk, role in self.dp["pieces"]:
                prog += [("run", role, self._dp_piece(d, k, bk)), ("reduce", bk, role)]
        prog.append(("join", "s1", "s2"))
        if dp:
            prog.append(("finish",))
        prog.append(("run", "s1", sgd))
        return prog, env

    def _streams(self):
        s1 = torch.cuda.current_stream()
        s2 = self._side()
        return {"s1": s1, "s2": s2 if s2 is not None else s1}

    def _host_op(self, op, S):
        if op[0] == "join":
            if S[op[1]] is not S[op[2]]:
                S[op[1]].wait_stream(S[op[2]])
        elif op[0] == "reduce":
            with torch.cuda.stream(S[op[2]]):
                self._dp_launch_reduce(op[1])
        elif op[0] == "finish":
            for w in self.dp["works"]:
                w.wait()
            self.dp["works"] = []

    def _run_program(self):
        """One eager step through the program (data parallel / forced chain; the warm-up and
        run_batch path of that mode), on the caller's current stream as s1."""
        prog, env = self._program()
        S = self._streams()
        self.opt.zero_grad()
        self.model._set_dtype()
        for op in prog:
            if op[0] == "run":
                with torch.cuda.stream(S[op[1]]):
                    op[2]()
            else:
                self._host_op(op, S)
        # The step's tensors are released here, once every piece is queued: a block returns to
        # the pool of the stream it was allocated on, and its next user there is ordered after
        # the other stream's use of it -- an s1 tensor read on s2 by the final join (s1 waits for
        # s2 before SGD), an s2 tensor read on s1 by the next step's first join (s2 waits for s1).
        # (Kept alive until the next step, they raised the eager path's peak by one step's env.)
        self.loss = env["loss"]
        env.clear()

    def _record_program(self):
        """Record each piece as one graph on its stream; a memory pool per stream, so a graph never
        reuses memory that a concurrently running graph of the other stream still holds.  The
        pieces' tensors stay referenced (env) for the life of the recording."""
        prog, env = self._program()
        S = {"s1": self.stream, "s2": self._side() or self.stream}
        pools = {"s1": torch.cuda.graph_pool_handle()}
        pools["s2"] = pools["s1"] if S["s2"] is S["s1"] else torch.cuda.graph_pool_handle()
        self.opt.zero_grad()
        self.model._set_dtype()
        rec = []
        for op in prog:
            if op[0] == "run":
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=S[op[1]], pool=pools[op[1]],
                                      capture_error_mode=CAPTURE_MODE):
                    op[2]()
                rec.append(("graph", op[1], g))
            else:
                rec.append(op)
        self._rec = rec
        self._rec_env = env
        self.loss = env["loss"]
        self.graph = next(o[2] for o in rec if o[0] == "graph")

    def _replay_program(self):
        S = self._streams()
        for op in self._rec:
            if op[0] == "graph":
                with torch.cuda.stream(S[op[1]]):
                    op[2].replay()
            else:
                self._host_op(op, S)

    # ---- data parallel: arena, buckets, deferred encoder backward ----------------------------
    def _bind(self):
        """Point the encoders' deferred-backward holders at THIS step's (several TrainSteps may
        share one model: ShapeGraphCache keeps one per frame size)."""
        if self.dp is not None:
            for e, d in zip((self.model.encoder, self.model.depth_encoder), self.dp["defers"]):
                e._cn_defer = d

    def _dp_setup(self):
        """Gradient arena and buckets: [RGB head + decoder], [depth head], then one bucket per
        encoder-backward segment of each encoder (RGB: [ASPP + layer4], layer3 halves, [layer2 +
        layer1 + stem]; depth: [ASPP + layer4], layer3, [layer2 + layer1 + stem]).  `pieces` =
        (holder, segment, bucket, stream role) in issue order: depth segment j, then RGB segment
        j -- each side's segments follow each other on its own stream."""
        from .encoder_fn import DeferredEncoderBwd
        m = self.model
        train = [p for p in self.params]
        tid = {id(p) for p in train}
        encs = [m.encoder, m.depth_encoder]
        defers = [DeferredEncoderBwd(e, None) for e in encs]
        enc_ids = {id(p) for e in encs for p in e.parameters()}
        dep_mods = [m.depth_similarity_weights, m.depth_gate, m.depth_reduce_channels, m.depth_bn,
                    m.depth_weights]
        dep_ids = {id(p) for mod in dep_mods for p in mod.parameters()}
        head_rgb = [p for p in train if id(p) not in enc_ids and id(p) not in dep_ids]
        head_dep = [p for p in train if id(p) in dep_ids]
        buckets = [head_rgb, head_dep]
        pieces = []
        for j in range(max(len(d.plan) for d in defers)):
            for d, role in ((defers[1], "s2"), (defers[0], "s1")):
                if j < len(d.plan):
                    pieces.append((d, j, len(buckets), role))
                    buckets.append([p for p in d.segment_params(j) if id(p) in tid])
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
        self.dp = {"buckets": buckets, "ranges": ranges, "pieces": pieces, "flat": flat,
                   "arena": arena, "views": views, "half": half, "works": [],
                   "head_live": [None, None], "defers": defers, "issued": 0,
                   "avg": bool(getattr(self, "coll", False)) and dist.get_backend(self.group) == "nccl"}
        self.flat = flat

    def _dp_head_bucket(self, k):
        """Head bucket k (0: RGB head + decoder, 1: depth head): copy the autograd gradients into
        the arena and ready the bucket for its all-reduce."""
        dp = self.dp
        if dp["head_live"][k] is None:   # which head parameters receive a gradient (static)
            dp["head_live"][k] = [p for p in dp["buckets"][k] if p.grad is not None]
        live = dp["head_live"][k]
        if live:
            torch._foreach_copy_([dp["views"][p] for p in live], [p.grad for p in live])
        self._dp_prepare_bucket(k)

    def _dp_piece(self, d, k, bk):
        def piece():
            d.run(k)
            self._dp_prepare_bucket(bk)
        return piece

    def _dp_prepare_bucket(self, k):
        """Device work that readies bucket k for its all-reduce: the 1/world pre-scale (sum of
        scaled = DataParallel's mean) and, for bf16 reduction, the cast.  On RCCL the bucket is
        reduced with ReduceOp.AVG instead: RCCL applies the 1/world factor inside its reduction
        kernel (a pre-multiplied sum), so the separate read + write pass over the 570 MB of
        gradients per step is gone; gloo has no AVG and keeps the pre-scale."""
        dp = self.dp
        a, b = dp["ranges"][k]
        if b == a:
            return
        if not dp["avg"]:
            nv.call("cn_scale", dp["flat"][a:].data_ptr(), b - a, 1.0 / self.world, nv.stream())
        if dp["half"] is not None:
            ops.cast_copy(dp["flat"][a:b].view(-1, 1), dp["half"][a:b].view(-1, 1))

    def _dp_launch_reduce(self, k):
        """Issue bucket k's all-reduce (async): RCCL waits for the work queued so far on the
        current stream and runs beside the pieces queued after it.  World 1 without collectives
        (forced chain): none."""
        dp = self.dp
        a, b = dp["ranges"][k]
        if b == a or not self.coll:
            return
        buf = dp["half"][a:b] if dp["half"] is not None else dp["flat"][a:b]
        op = dist.ReduceOp.AVG if dp["avg"] else dist.ReduceOp.SUM
        dp["works"].append(dist.all_reduce(buf, op=op, group=self.group, async_op=True))
        dp["issued"] += 1

    def _dp_sgd(self):
        """(Cast the reduced bf16 buckets back,) point the parameters' .grad at the arena, SGD."""
        dp = self.dp
        if dp["half"] is not None:
            ops.cast_copy(dp["half"].view(-1, 1), dp["flat"].view(-1, 1))
        live = set(id(p) for k in (0, 1) for p in (dp["head_live"][k] or []))
        for b_i, b in enumerate(dp["buckets"]):
            for p in b:
                if b_i > 1 or id(p) in live:
                    p.grad = dp["views"][p]
        self.opt.step()

    # ---- capture / replay ---------------------------------------------------------------------
    def _bn_counts(self):
        return {m: getattr(m, "_cn_nbt", 0) for m in self.model.modules()
                if isinstance(m, torch.nn.modules.batchnorm._BatchNorm)}

    def capture(self, warmup=2):
        """Run `warmup` eager iterations (they are real steps) on a side stream, then record."""
        if self.dp_mode and self.dp is None:
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
            if self.dp_mode or self._split_ok():
                self._record_program()
            else:
                self.graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(self.graph, stream=s, capture_error_mode=CAPTURE_MODE):
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

    def run_batch(self, rgb_a, rgb_b, dep_a, dep_b, gt_a, gt_b, lrs):
        """One EAGER iteration on inputs of any size (the reference's augmented batches change
        H, W every batch, so they cannot replay one recorded graph)."""
        if self.graphed and self.graph is not None:
            raise RuntimeError("run_batch is the eager path; build the TrainStep with graphed=False")
        if self.dp_mode and self.dp is None:
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
        if self.dp_mode and self.dp is None:
            self._dp_setup()
        self._bind()

        def once():
            self._counts()
            self.opt.refresh_lrs()
            if self.dp_mode:
                self._run_program()
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
        if self._rec is not None:
            self._replay_program()
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
