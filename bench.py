"""Throughput benchmark of the hot path: one training step of RGBDSegmentation_RAA
(forward of both frames x both modalities, co-attention, decoder, BCE+L1 loss, backward,
RCCL gradient all-reduce for N > 1, SGD step) on synthetic 473x473 RGB-D frame pairs,
batch 4 per GPU, bf16 compute (BASELINE.json configs[1]; configs[2] when launched on 8 GPUs).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...

Prints ONE JSON line (rank 0).  value = frame pairs per second over all ranks.
roofline: the implicit-GEMM MFMA kernel (every conv / linear / bmm of the step): algorithmic
FLOPs (2*M*N*K per launch) / measured launch time (HIP events on the launch stream over the
timed steps), against the 2.5 PFLOP/s dense bf16 MFMA peak of MI355X.
cpu_baseline: the oracle's CPU restatement (fp32 torch CPU, the reference's own op sequence)
timed on this host on a bounded sample (one B=2 fwd+bwd step at 473x473).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

MFMA_BF16_PEAK_TFLOPS = 2500.0   # MI355X dense bf16 (MI355X_MICROARCH.md)
MFMA_F32_PEAK_TFLOPS = 157.3
HBM_PEAK_GBS = 8000.0            # MI355X HBM3E (MI355X_MICROARCH.md)
# Index of the committed profiles the line cross-checks its live numbers against, with the source
# hash of the library they were taken with (tools/profile_index.py writes it after a profiling pass)
PROFILE_INDEX = os.path.join(REPO, "profiles", "current.json")


def committed_profile(kind):
    """(path, provenance) of the committed profile `kind` ("rocprof_stats", "coatt_trace", "pmc"):
    provenance = {"lib_source_hash" of the profiled library, "stale": whether the library loaded
    now was built from other sources -- then the committed numbers describe older kernels}."""
    try:
        with open(PROFILE_INDEX) as f:
            idx = json.load(f)
        path = os.path.join(REPO, idx[kind])
    except (OSError, KeyError, ValueError):
        return None, None
    try:
        from cosnet_amd import _native as nv
        now = nv.load().cn_build_source_hash().decode()
    except Exception:
        now = None
    return path, {"profiled_lib_source_hash": idx.get("lib_source_hash"), "loaded_lib_source_hash": now,
                  "stale": now != idx.get("lib_source_hash")}


def rocprof_avg_us(substr):
    """Average launch duration of a kernel family in the committed rocprofv3 --stats summary of
    this same bench command (the cross-check of the live HIP-event timing)."""
    path, prov = committed_profile("rocprof_stats")
    if path is None:
        return None
    try:
        import csv
        with open(path) as f:
            rows = [r for r in csv.DictReader(f) if substr in r["Name"]]
        n = sum(int(r["Calls"]) for r in rows)
        return dict({"avg_launch_us": sum(float(r["TotalDurationNs"]) for r in rows) / n / 1e3,
                     "launches": n, "source": os.path.relpath(path, REPO)}, **prov) if n else None
    except (OSError, KeyError, ValueError):
        return None


def coatt_trace():
    """Co-attention kernel time per training step / per configs[3] launch from the committed
    rocprofv3 --kernel-trace summary of this bench command (tools/coatt_trace_summary.py)."""
    path, prov = committed_profile("coatt_trace")
    if path is None:
        return None
    try:
        with open(path) as f:
            d = json.load(f)
        d["source"] = os.path.relpath(path, REPO) + ": " + d.get("source", "")
        d.update(prov)
        return d
    except (OSError, ValueError):
        return None


FLOP_PER_PAIR_473 = 4.1364e12    # SURVEY.md §8d (flop_counter on the reference graph)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=4, help="frame pairs per GPU")
    ap.add_argument("--size", type=int, default=473)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32", "fp8"],
                    help="fp8: e4m3 operands for the encoders' forward conv GEMMs (BASELINE "
                         "configs[4]; bf16 everywhere else)")
    ap.add_argument("--cpu-baseline", type=int, default=1, help="time the CPU oracle (rank 0)")
    ap.add_argument("--fp32-extra", type=int, default=1,
                    help="also time a few recorded fp32 steps (full-precision throughput beside "
                         "the bf16 headline; N = 1 only)")
    ap.add_argument("--fp8-extra", type=int, default=1,
                    help="also time a few recorded steps of BASELINE configs[4]'s per-GPU fp8 "
                         "workload (8 pairs; N = 1 only)")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--graph", type=int, default=1, help="replay the step as a HIP graph")
    ap.add_argument("--dp-chain", type=int, default=0,
                    help="1: run the data-parallel chain (arena, staged encoder backward, bucket "
                         "pre-scales) at N = 1 without collectives -- configs[2]'s per-rank step "
                         "timed on one GPU (the line says parallelism dp1-chain)")
    ap.add_argument("--grad-dtype", default="fp32", choices=["fp32", "bf16"],
                    help="data-parallel gradient buckets reduced in fp32 (default) or bf16")
    ap.add_argument("--dist-backend", default=None, choices=["nccl", "gloo"],
                    help="N > 1: nccl (RCCL, the default) or gloo (rehearse the multi-rank path on "
                         "one device, not a measurement).  N = 1 with --dp-chain 1 and nccl: a "
                         "world-1 RCCL process group with the chain's all-reduces really issued "
                         "(parallelism dp1-chain-rccl)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher / process-group plumbing only (no model, no GPU)")
    return ap.parse_args()


def pmc_traffic(family):
    """HBM traffic per launch of a kernel family from the committed rocprofv3 PMC summary
    (tools/pmc_run.sh + tools/pmc_summary.py over this bench's own eager step)."""
    path, prov = committed_profile("pmc")
    if path is None:
        return None
    try:
        with open(path) as f:
            d = json.load(f)
        e = dict(d["families"][family])
        e["source"] = os.path.relpath(path, REPO) + ": " + d["source"]
        e.update(prov)
        return e
    except (OSError, KeyError, ValueError):
        return None


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(size, reps=3):
    """The oracle's CPU restatement of the reference op sequence (fp32 torch CPU), timed on this
    host on bounded samples, median of `reps` runs each:
      train: one B=2 fwd+loss+bwd step at size x size (train mode needs B >= 2) -> the metric;
      c1:    one eval forward of a 240x320 pair (BASELINE configs[0]);
      c4:    test.py's N-reference loop (test.py:287-305): 5 eval forwards of the target with
             one reference each at size x size, once (configs[3])."""
    import statistics
    import torch
    from cosnet_amd.init_recipe import recipe_state_dict, synthetic_inputs
    import cosnet_amd as C
    from oracle.model_ref import RefModel, loss_bce_l1
    # the cores this process may actually use (the GPU box reports the whole host in
    # os.cpu_count() but grants a share: OMP_NUM_THREADS / the affinity mask)
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    threads = max(1, min(avail, int(os.environ.get("OMP_NUM_THREADS", avail))))
    torch.set_num_threads(threads)
    tmpl = C.build_model().state_dict()
    sd = recipe_state_dict(tmpl)
    ref = RefModel(sd, dtype=torch.float32)
    ra, rb, da, db, ga, gb = synthetic_inputs(2, size, size, seed=99)
    ts = []
    for _ in range(reps):
        for p in ref.p.values():
            p.grad = None
        t0 = time.perf_counter()
        x1, x2, _ = ref.forward(ra, rb, da, db)
        loss = loss_bce_l1(x1, ga) + loss_bce_l1(x2, gb)
        loss.backward()
        ts.append(time.perf_counter() - t0)
    dt = statistics.median(ts)
    evr = RefModel(sd, dtype=torch.float32, requires_grad=False)
    evr.training = False
    c1 = synthetic_inputs(1, 240, 320, seed=77)
    t1 = []
    with torch.no_grad():
        for _ in range(reps):
            t0 = time.perf_counter()
            evr.forward(*c1[:4])
            t1.append(time.perf_counter() - t0)
    n_ref = 5
    q = synthetic_inputs(n_ref, size, size, seed=5)
    with torch.no_grad():
        t0 = time.perf_counter()
        for i in range(n_ref):  # target re-encoded per reference, as test.py:287-293 does
            evr.forward(q[0][:1], q[1][i:i + 1], q[2][:1], q[3][i:i + 1])
        t4 = time.perf_counter() - t0
    return {"value": 2.0 / dt, "unit": "frame-pairs/s", "cores": torch.get_num_threads(),
            "kind": "port", "cpu": _cpu_model(),
            "sample": "median of %d train steps (fwd+loss+bwd), B=2 pairs at %dx%d, fp32 torch CPU "
                      "restatement of the reference op sequence (oracle/model_ref.py): %s s" % (
                          reps, size, size, ", ".join("%.2f" % t for t in ts)),
            "c1_eval_240x320_pairs_per_s": 1.0 / statistics.median(t1),
            "c1_sample": "median of %d eval forwards, 1 pair 240x320: %s s" % (
                reps, ", ".join("%.2f" % t for t in t1)),
            "c4_targets_per_s": 1.0 / t4,
            "c4_sample": "test.py N-reference loop, 1 target x %d references at %dx%d (5 eval "
                         "forwards): %.2f s" % (n_ref, size, size, t4)}


def coattention_roofline(dev, n=5, hw=3600, c=256, iters=20):
    """Fused co-attention kernel (cn_coatt_fused_fwd: S = Va_t Vb^T, both softmax directions and
    both gathers without materialising S) on the inference shape of BASELINE configs[3]: one
    target + 5 reference frames at 473x473 -> n = 5 pairs of 60x60x256 bf16 features.
    Algorithmic work 3 x 2 HW^2 C per pair (the kernel executes 4 x, S is
    recomputed per direction), timed with HIP events around a HIP graph of `iters` launches (as
    the step runs them: recorded, no host gaps; the launch's workspace counter reset included) and
    as eager back-to-back calls, both in a settled clock state."""
    import torch
    from cosnet_amd import ops
    g = torch.Generator(device="cpu").manual_seed(3)
    vat, va, vb = [(torch.randn((n * hw, c), generator=g) * 0.7).to(torch.bfloat16).to(dev)
                   for _ in range(3)]
    za = torch.empty_like(va)
    zb = torch.empty_like(va)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            ops.coatt_fused(vat, va, vb, n, hw, za, zb)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        for _ in range(iters):
            ops.coatt_fused(vat, va, vb, n, hw, za, zb)

    def replay():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        graph.replay()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e-3 / iters

    def eager():
        # the same launches issued eagerly back to back (each call's host work -- workspace
        # query, allocation, counter memset, launch -- included): an un-recorded caller's view
        with torch.cuda.stream(s):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record(s)
            for _ in range(iters):
                ops.coatt_fused(vat, va, vb, n, hw, za, zb)
            e1.record(s)
            torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e-3 / iters

    # settle: after the gap this line's setup leaves, the kernel speeds up for tens of ms (170 ->
    # 145 us per launch over ~30 ms, graph or eager alike) while the reported gfx / memory clocks
    # stay put and the socket power climbs (profiles/r06_clock_probe.txt) -- a warm-up below what
    # amdsmi reports; replay until two replays in a row agree within 1 %
    first = prev = replay()
    settle = 1
    while settle < 60:
        cur = replay()
        settle += 1
        if abs(cur - prev) <= 0.01 * prev:
            break
        prev = cur
    ts, te = [], []
    for _ in range(5):   # graph and eager interleaved, so neither sees a different clock state
        ts.append(replay())
        te.append(eager())
    t = sorted(ts)[2]
    t_eager = sorted(te)[2]
    # release the recording and its private memory pool before the extra lines run (left alive,
    # the fp8 extra line measured 152 instead of 166 frame-pairs/s after it)
    del graph
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    alg = 3 * 2.0 * n * hw * hw * c
    return {"bound": "mfma", "kernel": "coatt_q48_k (48 query rows per wave, stream-K over the CUs; flash-style, S never in HBM)",
            "workload": "%d pairs x HW %d x C %d bf16 (configs[3]: 1 target + 5 refs, 473x473)" % (n, hw, c),
            "achieved": alg / t / 1e12, "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": alg / t / 1e12 / MFMA_BF16_PEAK_TFLOPS,
            "executed_tflops": 4 / 3 * alg / t / 1e12, "us_per_launch": t * 1e6,
            "timing": "kernel-only: HIP events around a recorded graph of %d launches, median of 5 "
                      "interleaved with the eager timing, after %d settling replays (the first: "
                      "%.1f us per launch)" % (iters, settle, first * 1e6),
            "us_per_launch_eager": t_eager * 1e6, "frac_eager": alg / t_eager / 1e12 / MFMA_BF16_PEAK_TFLOPS}


def extra_line(dev, B, S, kind, steps=5, warmup=2):
    """A second precision beside the bf16 headline, the same recorded train step timed over
    `steps` replays after `warmup`:
      fp32 -- every GEMM on the f32 MFMA (157 TFLOP/s peak), B pairs;
      fp8  -- BASELINE configs[4]'s per-GPU step (8 pairs, 64 over 8 GPUs): e4m3 forward convs,
              e5m2 dgrads, bf16 weight gradients and co-attention training kernels."""
    import torch
    import cosnet_amd as C
    from cosnet_amd.init_recipe import recipe_state_dict, synthetic_inputs
    from cosnet_amd.optim import SGD, reference_param_groups
    from cosnet_amd.train_step import TrainStep
    m = C.build_model(torch.float32 if kind == "fp32" else torch.bfloat16)
    m.load_state_dict(recipe_state_dict(m.state_dict()))
    if kind == "fp8":
        m.set_fp8(True)
    m.encoder.main_classifier.requires_grad_(False)
    m = m.to(dev).train()
    g0, g1 = reference_param_groups(m)
    opt = SGD([g0, g1], [2.5e-6, 2.5e-3], momentum=0.9, weight_decay=5e-4)
    st = TrainStep(m, opt, B, S, graphed=True)
    st.load(*[t.to(dev) for t in synthetic_inputs(B, S, S, seed=1234)])
    st.capture(warmup=warmup)
    st([2.5e-6, 2.5e-3])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = st([2.5e-6, 2.5e-3])
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    out = {"value": B * steps / dt, "unit": "frame-pairs/s", "dtype": kind, "batch": B,
           "steps": steps, "ms_per_step": dt / steps * 1e3, "loss": float(loss.item()),
           "model_tflops_per_s": B * steps * FLOP_PER_PAIR_473 / dt / 1e12 if S == 473 else None}
    if kind == "fp32":
        out["peak_tflops"] = MFMA_F32_PEAK_TFLOPS
    # the model and its step hold reference cycles (encoder <-> deferred-backward holder, the
    # recording's tensors): collect them, or each extra line leaves ~10 GB reserved
    # (profiles/r06_bench_order_probe.txt)
    del st, opt, m
    import gc
    gc.collect()
    torch.cuda.empty_cache()
    return out


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _launch_ranks(n, argv):
    """--gpus N outside a torch.distributed launcher: start one rank per GPU as a CHILD
    `torch.distributed.run` (nothing in this process has touched the GPU, and it is never
    exec-replaced); rank 0's JSON line reaches stdout through the inherited descriptor.
    Reference: train.py:491-496 (DataParallel over --gpus), here one process per GPU."""
    import subprocess
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + list(argv)
    return subprocess.call(cmd, env=env)


def dry_run(args, world, rank):
    """--dry-run: the launcher / process-group / max-over-ranks timing plumbing of this bench
    without the model (CPU gloo; used by tests/test_cli.py to check the N-rank launch)."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")
        dist.barrier()
    t0 = time.perf_counter()
    time.sleep(0.01 * (rank + 1))
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = t.item()
    if rank == 0:
        print(json.dumps({"metric": "dry-run (launcher plumbing only)", "value": None,
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "max_rank_seconds": dt,
                          "config": {"parallelism": "dp%d" % world}}), file=_json_out(), flush=True)
    if world > 1:
        dist.destroy_process_group()


_JSON_OUT = None


def _json_out():
    return _JSON_OUT or sys.stdout


def _claim_stdout():
    """The JSON line is the only thing this process writes to stdout: native libraries print to
    fd 1 too (RCCL's version banner at communicator init), so fd 1 becomes a copy of stderr and
    the line goes to a private duplicate of the original stdout."""
    global _JSON_OUT
    try:
        sys.stdout.flush()
        _JSON_OUT = os.fdopen(os.dup(1), "w")
        os.dup2(2, 1)
    except OSError:
        _JSON_OUT = None


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return _launch_ranks(args.gpus, sys.argv[1:])
    _claim_stdout()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus and "WORLD_SIZE" in os.environ:
        print("[bench] note: --gpus %d but WORLD_SIZE=%d; the launcher's world size is used"
              % (args.gpus, world), file=sys.stderr)
    rank = int(os.environ.get("RANK", "0"))
    if args.dry_run:
        return dry_run(args, world, rank)
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = args.dist_backend or "nccl"
    if backend == "gloo":   # rehearsal: every rank on device 0
        local = 0
    # world-1 RCCL chain: configs[2]'s per-rank step with its collectives issued on a real
    # RCCL communicator (one rank, this device)
    rccl1 = world == 1 and args.dp_chain and args.dist_backend == "nccl"
    if world > 1 or rccl1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        init = {} if world > 1 else {"init_method": "tcp://127.0.0.1:%d" % _free_port(),
                                     "world_size": 1, "rank": 0}
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), **init)
        else:
            dist.init_process_group("gloo", **init)
    dev = torch.device("cuda", local)

    import cosnet_amd as C
    from cosnet_amd import ops
    from cosnet_amd.init_recipe import recipe_state_dict, synthetic_inputs
    from cosnet_amd.optim import SGD, lr_poly, reference_param_groups
    from cosnet_amd.train_step import TrainStep

    dtype = torch.float32 if args.dtype == "fp32" else torch.bfloat16
    torch.manual_seed(1234)
    model = C.build_model(dtype)
    model.load_state_dict(recipe_state_dict(model.state_dict()))
    if args.dtype == "fp8":
        model.set_fp8(True)
    # encoder.main_classifier only produces `labels`, which never enters the loss
    # (SURVEY.md §3.3): it receives no gradient in the reference either.
    model.encoder.main_classifier.requires_grad_(False)
    model = model.to(dev).train()
    g0, g1 = reference_param_groups(model)
    opt = SGD([g0, g1], [0.0, 0.0], momentum=0.9, weight_decay=5e-4)

    B, S = args.batch, args.size
    step = TrainStep(model, opt, B, S, graphed=bool(args.graph), grad_dtype=args.grad_dtype,
                     dp_chain=bool(args.dp_chain), collectives=bool(rccl1))
    step.load(*[t.to(dev) for t in synthetic_inputs(B, S, S, seed=1234 + rank)])
    max_iter = 10000

    def lrs(i):
        lr = lr_poly(2.5e-4, i, max_iter, 0.9, 0)
        return [0.01 * lr, 10 * lr]                  # train.py:171-172

    def log(msg):
        if rank == 0:
            print("[bench] " + msg, file=sys.stderr, flush=True)

    # warmup: the first (eager) iterations happen inside capture(); the rest are replays
    prof = ops.GemmProfile() if not args.no_roofline else None
    t1 = time.perf_counter()
    nw = max(1, min(args.warmup, 2))
    opt.set_lrs(lrs(0))
    step.capture(warmup=nw)
    torch.cuda.synchronize()
    log("capture + %d eager warmup steps: %.1f s" % (nw, time.perf_counter() - t1))
    for i in range(nw, args.warmup):
        t1 = time.perf_counter()
        step(lrs(i))
        torch.cuda.synchronize()
        log("warmup step %d: %.1f ms" % (i, (time.perf_counter() - t1) * 1e3))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if prof and not args.graph:
        prof.__enter__()
    host = []
    for i in range(args.steps):
        th = time.perf_counter()
        loss = step(lrs(args.warmup + i))
        host.append(time.perf_counter() - th)
    if prof and not args.graph:
        prof.__exit__()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = t.item()
    pairs = B * world * args.steps
    out = {
        "metric": "frame-pairs/sec (fwd+bwd) at 473x473 RGBD",
        "value": pairs / dt,
        "unit": "frame-pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        # host time inside step() per step (issuing the recorded graphs / the eager kernels): the
        # mean over the timed steps, and the first one (issued onto an idle device, so no queue
        # back-pressure is in it)
        "host_issue_ms_per_step": sum(host) / args.steps * 1e3,
        "host_issue_ms_first": host[0] * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic (seeded U[0,255) BGR-mean / depth, blob masks; name-keyed random-init weights)",
        "config": {"workload": "RGBDSegmentation_RAA train step (fwd+loss+bwd+SGD), %dx%d, "
                               "batch %d pairs/GPU" % (S, S, B),
                   "model": "RGBDSegmentation_RAA(Bottleneck,[3,4,23,3],[3,4,6,3],1)",
                   "global_batch": B * world, "image_hw": [S, S],
                   "parallelism": "dp%d" % world + ("-chain" if args.dp_chain and world == 1 else "")
                                  + ("-rccl" if rccl1 else ""),
                   "grad_reduce": "%s buckets overlapped with the encoder backward" % args.grad_dtype
                   if world > 1 or rccl1 else None,
                   "loss": float(loss.item())},
        "model_tflops_per_s": pairs * FLOP_PER_PAIR_473 / dt / 1e12 if S == 473 else None,
    }
    if prof and args.graph:
        # ROCm graphs cannot carry timing events: time the GEMM launches of one more step,
        # run eagerly right after the timed replays (same kernels, shapes and weights)
        # (encoders on one stream here: events around a launch that overlaps the other
        # stream's kernels would charge it their time)
        # The depth parameters' AccumulateGrad nodes were created on the second stream; moving
        # the depth encoder to the main stream for this one step is a deliberate stream change,
        # so autograd's mismatch warning is silenced for it (and restored after).
        conc = getattr(model, "concurrent_encoders", False)
        model.concurrent_encoders = False
        warn = torch.autograd.graph.set_warn_on_accumulate_grad_stream_mismatch
        warn(False)
        # hold the device with a spin kernel while the host queues the whole eager step, so the
        # events bracket back-to-back kernels (host launch gaps would otherwise be timed too)
        torch.cuda.synchronize()
        torch.cuda._sleep(int(0.4 * 2.0e9))
        with prof:
            step.eager(lrs(args.warmup + args.steps))
        torch.cuda.synchronize()
        warn(True)
        model.concurrent_encoders = conc
    if prof:
        n, fl, kt = prof.summary()
        nbytes = prof.algorithmic_bytes()
        # the flash co-attention launches are reported on their own (roofline_coattention_train)
        fn_, ffl, ft, fb = [a + b for a, b in zip(prof.select("coatt_flash_fwd"),
                                                 prof.select("coatt_flash_bwd"))]
        n, fl, kt, nbytes = n - fn_, fl - ffl, kt - ft, nbytes - fb
        if args.graph:  # one eager step: scale to the timed steps
            n, fl, kt, nbytes = n * args.steps, fl * args.steps, kt * args.steps, nbytes * args.steps
        peak = MFMA_BF16_PEAK_TFLOPS if dtype == torch.bfloat16 else MFMA_F32_PEAK_TFLOPS
        ach = fl / kt / 1e12
        pmc = pmc_traffic("gemm_kernel")
        out["roofline"] = {"bound": "mfma", "kernel": "gemm_kernel (implicit-GEMM conv/bmm)",
                           "achieved": ach, "peak": peak, "unit": "TFLOP/s", "frac": ach / peak,
                           "traffic": pmc["traffic_bytes_per_launch"] if pmc else None,
                           "traffic_unit": "HBM bytes per launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE)",
                           "traffic_source": pmc["source"] if pmc else None,
                           "traffic_stale": pmc["stale"] if pmc else None,
                           "algorithmic_bytes_per_launch": nbytes / n,
                           "event_avg_launch_us": kt / n * 1e6,
                           "rocprof": rocprof_avg_us("gemm_kernel"),
                           "launches_per_step": n / args.steps,
                           "gemm_time_frac_of_step": kt / dt,
                           "gemm_tflop_per_step": fl / args.steps / 1e12}
        # the HW x HW affinity bmm S = (Va W^T) Vb^T (rgbd_segmentation_RAA.py:160,213): it writes
        # the fp32 S to HBM, so its roofline is HBM bandwidth
        an, afl, at, ab = prof.select("affinity")
        if an:
            out["roofline_affinity"] = {
                "bound": "hbm", "kernel": "gemm_kernel, S = Va_t . Vb^T with fp32 S (B*HW x HW)",
                "achieved": ab / at / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": ab / at / 1e9 / HBM_PEAK_GBS, "tflops": afl / at / 1e12,
                "mfma_frac": afl / at / 1e12 / peak, "launches_per_step": an / (1 if args.graph else args.steps),
                "bytes_per_launch": ab / an, "us_per_launch": at / an * 1e6}
        if fn_:
            # training co-attention (both modalities): flash forward + the two backward kernels,
            # algorithmic FLOPs (ops.coatt_flash_fwd / coatt_flash_bwd tags)
            sc = 1 if args.graph else args.steps
            out["roofline_coattention_train"] = {
                "bound": "mfma", "kernel": "coatt_flash fwd (S never in HBM, LSE kept) + dVa_t + PV backward",
                "achieved": ffl / ft / 1e12, "peak": peak, "unit": "TFLOP/s", "frac": ffl / ft / 1e12 / peak,
                "launches_per_step": fn_ / sc, "us_per_step": ft / sc * 1e6,
                "fwd_tflops": prof.select("coatt_flash_fwd")[1] / max(prof.select("coatt_flash_fwd")[2], 1e-12) / 1e12,
                "bwd_tflops": prof.select("coatt_flash_bwd")[1] / max(prof.select("coatt_flash_bwd")[2], 1e-12) / 1e12,
                "algorithmic_gflop_per_step": ffl / sc / 1e9}
            tr = coatt_trace()
            if tr:
                us = tr["train_us_per_step"]
                out["roofline_coattention_train"]["rocprof"] = {
                    "us_per_step": us, "frac": ffl / sc / (us * 1e-6) / 1e12 / peak, "source": tr["source"],
                    "stale": tr["stale"]}
    log("timed: %.1f ms/step" % (dt / args.steps * 1e3))
    if args.fp32_extra and dtype == torch.bfloat16 and world == 1 and not args.no_roofline:
        log("fp32 extra ...")
        out["fp32_extra"] = extra_line(dev, B, S, "fp32")
    if args.fp8_extra and args.dtype == "bf16" and world == 1 and not args.no_roofline and S == 473:
        log("fp8 extra (configs[4] per-GPU batch 8) ...")
        out["fp8_extra"] = extra_line(dev, 8, S, "fp8")
    # after the extra lines (round 5 saw the fp8 line at 152 instead of 166 frame-pairs/s with
    # the configs[3] recording run first; round 6's probe no longer reproduces it, and the
    # recording is released before returning)
    if prof and dtype == torch.bfloat16 and S == 473:
        out["roofline_coattention"] = rc = coattention_roofline(dev)
        tr = coatt_trace()
        if tr and tr.get("configs3_us_per_launch"):
            us = tr.get("configs3_us_per_launch_timed") or tr["configs3_us_per_launch"]
            alg = rc["achieved"] * rc["us_per_launch"] * 1e-6 * 1e12
            rc["rocprof"] = {"us_per_launch": us, "frac": alg / (us * 1e-6) / 1e12 / MFMA_BF16_PEAK_TFLOPS,
                             "source": tr["source"], "stale": tr["stale"]}
    out["build"] = __import__("cosnet_amd._native", fromlist=["build_info"]).build_info()
    if rank == 0 and args.cpu_baseline and world == 1:
        log("cpu baseline ...")
        try:
            out["cpu_baseline"] = cpu_baseline(S)
        except Exception as e:  # report, never hide
            out["cpu_baseline"] = {"error": repr(e)}
    if rank == 0:
        print(json.dumps(out), file=_json_out(), flush=True)
    if world > 1 or rccl1:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
