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

Data parallel (world > 1): the graph ends by packing every gradient into one flat fp32 buffer;
the buffer is averaged with ONE RCCL all-reduce (ReduceOp.AVG, the DDP gradient semantics) and
the SGD kernel reads its gradients straight out of it.  BN running statistics stay per rank
during training (train-mode BN normalises with batch statistics, so they never enter the
step); sync_buffers() broadcasts rank 0's before evaluation or checkpointing.
"""
import torch
import torch.distributed as dist

from . import functions as fn


class TrainStep:
    """`size` = H (square frames) or (H, W); `batch` = frame pairs on this rank."""

    def __init__(self, model, opt, batch, size, l1_weight=0.8, graphed=True, group=None):
        self.model, self.opt = model, opt
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
        if self.world == 1:
            self.opt.step()
        else:
            self._pack()

    def _flat_views(self):
        """fp32 flat gradient buffer + one view per parameter with the parameter's strides."""
        n = sum(p.numel() for p in self.params)
        self.flat = torch.zeros((n,), dtype=torch.float32, device=self.params[0].device)
        self.views = []
        off = 0
        for p in self.params:
            v = self.flat[off:off + p.numel()].as_strided(p.shape, p.stride())
            self.views.append(v)
            off += p.numel()

    def _pack(self):
        grads, views = [], []
        for p, v in zip(self.params, self.views):
            if p.grad is not None:
                grads.append(p.grad)
                views.append(v)
        torch._foreach_copy_(views, grads)

    def _after_pack(self):
        """world > 1: average the packed gradients and step SGD on them (eager, two calls)."""
        if dist.get_backend(self.group) == "nccl":   # RCCL averages in the collective
            dist.all_reduce(self.flat, op=dist.ReduceOp.AVG, group=self.group)
        else:                                           # gloo (CPU-side tests): no AVG op
            dist.all_reduce(self.flat, group=self.group)
            self.flat.mul_(1.0 / self.world)
        saved = [p.grad for p in self.params]
        for p, v in zip(self.params, self.views):
            if p.grad is not None:
                p.grad = v
        self.opt.step()
        for p, g in zip(self.params, saved):
            p.grad = g

    # ---- capture / replay ---------------------------------------------------------------------
    def _bn_counts(self):
        return {m: getattr(m, "_cn_nbt", 0) for m in self.model.modules()
                if isinstance(m, torch.nn.modules.batchnorm._BatchNorm)}

    def capture(self, warmup=2):
        """Run `warmup` eager iterations (they are real steps) on a side stream, then record."""
        if self.world > 1:
            self._flat_views()
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
        torch.cuda.synchronize()
        self.opt.reserve()
        self.opt.freeze_for_capture()
        self.opt.refresh_lrs()
        torch.cuda.synchronize()
        before = self._bn_counts()
        self.graph = torch.cuda.CUDAGraph()
        self._capturing = True
        try:
            with torch.cuda.graph(self.graph, stream=s):
                self._body()
        finally:
            self._capturing = False
        self._graph_loss = self.loss
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
        if self.world > 1 and self.flat is None:
            self._flat_views()
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
        def once():
            self._counts()
            self.opt.refresh_lrs()
            self._body()
            if self.world > 1:
                self._after_pack()
        self._on_stream(once)

    def __call__(self, lrs):
        """One iteration on the loaded inputs with learning rates `lrs` (one per group)."""
        self.opt.set_lrs(lrs)
        if self.graph is None:
            self._eager_once()
            return self.loss
        self.opt.refresh_lrs()
        self._counts()
        self.graph.replay()
        self.loss = self._graph_loss
        self._mem(" After forward")
        self._mem(" After backward")
        # the replay updated the fp32 masters AND their compute-dtype copies in place (cn_sgd):
        # the weight cache stays valid
        for m, d in self._nbt_delta.items():
            m._cn_nbt = getattr(m, "_cn_nbt", 0) + d
        if self.world > 1:
            self._after_pack()
        return self.loss

    def sync_buffers(self, src=0):
        """Broadcast rank `src`'s BN running statistics (before eval / checkpoint)."""
        if self.world > 1:
            for b in self.model.buffers():
                dist.broadcast(b, src, group=self.group)
