"""The HIP-graph replayed training step (cosnet_amd/train_step.py) against the eager step."""
import pytest
import torch

import cosnet_amd as C
from cosnet_amd import ops
from cosnet_amd.init_recipe import recipe_state_dict, synthetic_inputs
from cosnet_amd.optim import SGD, lr_poly, reference_param_groups
from cosnet_amd.train_step import TrainStep


def _setup(cuda, dtype, graphed, b=2, s=65, split=False, chain=False, coll=False):
    torch.manual_seed(0)
    fp8 = dtype == "fp8"
    m = C.build_model(torch.bfloat16 if fp8 else dtype)
    m.load_state_dict(recipe_state_dict(m.state_dict()))
    if fp8:
        m.set_fp8(True)
    m.encoder.main_classifier.requires_grad_(False)
    m = m.to(cuda).train()
    g0, g1 = reference_param_groups(m)
    opt = SGD([g0, g1], [0.0, 0.0])
    st = TrainStep(m, opt, b, s, graphed=graphed, split_graphs=split, dp_chain=chain, collectives=coll)
    st.load(*[t.to(cuda) for t in synthetic_inputs(b, s, s, seed=5)])
    return m, st


def _lrs(i):
    lr = lr_poly(2.5e-4, i, 100, 0.9, 0)
    return [0.01 * lr, 10 * lr]  # train.py:171-172


def _bufs(st):
    return [st.opt.state[id(p)]["momentum_buffer"] for p in st.params if id(p) in st.opt.state]


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["one", "split", "chain"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, "fp8"])
def test_graph_step_matches_eager(cuda, dtype, mode):
    """Graph replays follow the eager trajectory BIT FOR BIT: every reduction of the step is a
    fixed-order sum (no float atomics; the co-attention's stream-K counters are memset nodes
    that only order the merge, not its sum), so two eager runs are bitwise
    identical, and so is the replayed graph -- losses, every SGD momentum buffer (the running
    sum of each parameter's gradients, so a gradient contribution missing from the recording
    shows up) and the BN running statistics.  mode "one": the step as one recorded graph; "split":
    one-stream graphs per phase and stream (TrainStep split_graphs, the default); "chain": the
    data-parallel chain (gradient arena, segment-by-segment encoder backward, bucket pre-scales)
    forced at world 1, eager against its own recording.  fp8: configs[4]'s per-GPU path (e4m3
    forward convs, e5m2 dgrads, delayed scaling state carried from step to step)."""
    if dtype == "fp8" and mode == "one":
        pytest.skip("fp8 covered by the split / chain recordings")
    split, chain = mode == "split", mode == "chain"
    runs = [_setup(cuda, dtype, graphed=g, split=split and g, chain=chain) for g in (False, False, True)]
    for _, st in runs:
        st.opt.set_lrs(_lrs(0))
        st.capture(warmup=2)
    assert (runs[2][1]._rec is not None) == (split or chain)
    losses = [[], [], []]
    for i in range(2):
        for r, (_, st) in enumerate(runs):
            losses[r].append(float(st(_lrs(2 + i))))
    torch.cuda.synchronize()
    assert losses[0] == losses[1] == losses[2], losses
    b0, b1, b2 = (_bufs(st) for _, st in runs)
    assert len(b0) == len(b2) > 300
    for k, (x0, x1, x2) in enumerate(zip(b0, b1, b2)):
        assert torch.equal(x0, x1), (k, tuple(x0.shape), "eager runs differ")
        assert torch.equal(x0, x2), (k, tuple(x0.shape), "graph differs from eager")
    sde, sdg = runs[0][0].state_dict(), runs[2][0].state_dict()
    for k in sde:
        if k.endswith("num_batches_tracked"):
            assert int(sde[k]) == int(sdg[k]), k
        elif k.endswith("running_mean") or k.endswith("running_var"):
            assert torch.equal(sde[k], sdg[k]), k
    # the eager path must see the weights the replays produced (weight cache invalidated)
    me, mg, sg = runs[0][0], runs[2][0], runs[2][1]
    with torch.no_grad():
        xe = me(sg.rgb_a, sg.rgb_b, sg.dep_a, sg.dep_b)[0]
        xg = mg(sg.rgb_a, sg.rgb_b, sg.dep_a, sg.dep_b)[0]
    assert torch.equal(xe, xg)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_dp_chain_tracks_single_process_step(cuda, dtype):
    """The data-parallel chain at world 1 computes the single-process step's gradients: its
    encoder backward runs segment by segment (each segment's weight gradients grouped at its end
    instead of the whole encoder's at the end), so the grouped launches differ and with them the
    fp32 summation order of some weight gradients -- same math, bounded difference after two
    recorded steps."""
    runs = [_setup(cuda, dtype, graphed=True, split=True, chain=c) for c in (False, True)]
    for _, st in runs:
        st.opt.set_lrs(_lrs(0))
        st.capture(warmup=1)
    losses = [[float(st(_lrs(1 + i))) for i in range(2)] for _, st in runs]
    torch.cuda.synchronize()
    tol = 1e-4 if dtype == torch.float32 else 2e-2
    for a, b in zip(*losses):
        assert abs(a - b) <= tol * abs(a), losses
    b0, b1 = _bufs(runs[0][1]), _bufs(runs[1][1])
    assert len(b0) == len(b1) > 300
    num = sum(float((x - y).double().square().sum()) for x, y in zip(b0, b1))
    den = sum(float(x.double().square().sum()) for x in b0)
    assert (num / den) ** 0.5 <= (1e-3 if dtype == torch.float32 else 5e-2), (num / den) ** 0.5


@pytest.mark.gpu
def test_rccl_world1_chain_tracks_single_process_step_473(cuda):
    """configs[2]'s per-rank step (473x473, 4 pairs, bf16, recorded) through a REAL RCCL
    communicator: a world-1 "nccl" process group, the positive-count all-reduce and every
    bucket's async all-reduce issued from its piece's stream between the graph replays and
    waited on before SGD (TrainStep collectives=True) -- against the single-process step, with
    the bounds of test_dp_chain_tracks_single_process_step (bf16)."""
    import socket
    import torch.distributed as dist
    if dist.is_initialized():
        pytest.skip("a process group is already initialised in this process")
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port, world_size=1, rank=0,
                            device_id=cuda)
    try:
        assert dist.get_backend() == "nccl"
        runs = [_setup(cuda, torch.bfloat16, graphed=True, b=4, s=473, split=True, chain=c, coll=c)
                for c in (False, True)]
        single, chain = runs[0][1], runs[1][1]
        assert not single.coll and chain.coll and chain.dp_mode and chain.world == 1
        for _, st in runs:
            st.opt.set_lrs(_lrs(0))
            st.capture(warmup=1)
        assert chain._rec is not None and any(op[0] == "reduce" for op in chain._rec)
        issued0 = chain.dp["issued"]
        losses = [[float(st(_lrs(1 + i))) for i in range(2)] for _, st in runs]
        torch.cuda.synchronize()
        nb = sum(1 for a, b in chain.dp["ranges"] if b > a)
        assert chain.dp["issued"] - issued0 == 2 * nb, (chain.dp["issued"], issued0, nb)
        assert chain.dp["works"] == []
        for a, b in zip(*losses):
            assert abs(a - b) <= 2e-2 * abs(a), losses
        b0, b1 = _bufs(single), _bufs(chain)
        assert len(b0) == len(b1) > 300
        num = sum(float((x - y).double().square().sum()) for x, y in zip(b0, b1))
        den = sum(float(x.double().square().sum()) for x in b0)
        assert (num / den) ** 0.5 <= 5e-2, (num / den) ** 0.5
        assert all(torch.isfinite(x).all() for x in b1)
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_eager_after_graph_keeps_graph_tables(cuda):
    """An eager step after recording must not disturb the recorded SGD tables."""
    m1, s1 = _setup(cuda, torch.bfloat16, graphed=True)
    m2, s2 = _setup(cuda, torch.bfloat16, graphed=True)
    for st in (s1, s2):
        st.opt.set_lrs(_lrs(0))
        st.capture(warmup=1)
    s1(_lrs(1))
    s2(_lrs(1))
    prof = ops.GemmProfile()
    with prof:
        s1.eager(_lrs(2))
    s2.eager(_lrs(2))
    l1 = float(s1(_lrs(3)))
    l2 = float(s2(_lrs(3)))
    torch.cuda.synchronize()
    n, fl, t = prof.summary()
    assert n > 100 and fl > 0 and 0 < t < 1.0
    assert abs(l1 - l2) <= 1e-5 * abs(l1)


@pytest.mark.gpu
def test_two_stream_encoders_match_one_stream(cuda):
    """The depth encoder on its own stream (forward and, through autograd, backward; a parallel
    branch of the recorded graph) gives the step BIT-identical results to running both
    encoders on one stream: the kernels are deterministic, only their overlap changes."""
    runs = [_setup(cuda, torch.bfloat16, graphed=True) for _ in range(2)]
    runs[1][0].concurrent_encoders = False
    for _, st in runs:
        st.opt.set_lrs(_lrs(0))
        st.capture(warmup=1)
    losses = [[float(st(_lrs(1 + i))) for i in range(2)] for _, st in runs]
    torch.cuda.synchronize()
    assert losses[0] == losses[1], losses
    for k, (x0, x1) in enumerate(zip(_bufs(runs[0][1]), _bufs(runs[1][1]))):
        assert torch.equal(x0, x1), (k, tuple(x0.shape))
    p0 = [p.detach() for p in runs[0][0].parameters()]
    p1 = [p.detach() for p in runs[1][0].parameters()]
    assert all(torch.equal(a, b) for a, b in zip(p0, p1))


def test_shape_graph_cache_matches_eager(cuda):
    """ShapeGraphCache (train.py --dataset sbmrgbd: the frame size changes every batch): sizes
    seen twice are recorded and replayed, others run eagerly; the loss trajectory and the final
    parameters equal a plain eager run of the same batches (same kernels, same order: bitwise)."""
    import cosnet_amd as C
    from cosnet_amd.init_recipe import recipe_state_dict, synthetic_inputs
    from cosnet_amd.optim import SGD, reference_param_groups
    from cosnet_amd.train_step import ShapeGraphCache, TrainStep

    def model():
        m = C.build_model(torch.bfloat16)
        m.load_state_dict(recipe_state_dict(m.state_dict()))
        m.encoder.main_classifier.requires_grad_(False)
        m = m.to(cuda).train()
        g0, g1 = reference_param_groups(m)
        return m, SGD([g0, g1], [0.0, 0.0], momentum=0.9, weight_decay=5e-4)

    sizes = [(65, 81), (73, 57), (65, 81), (73, 57), (65, 81), (49, 65), (73, 57)]
    batches = [[t.to(cuda) for t in synthetic_inputs(2, h, w, seed=50 + i)] for i, (h, w) in enumerate(sizes)]
    lrs = [2.5e-6, 2.5e-3]
    m1, o1 = model()
    cache = ShapeGraphCache(m1, o1, 2, capacity=4, min_hits=2)
    l1 = [float(cache(*b, lrs).item()) for b in batches]
    m2, o2 = model()
    eager = TrainStep(m2, o2, 2, sizes[0], graphed=False)
    l2 = [float(eager.run_batch(*b, lrs).item()) for b in batches]
    torch.cuda.synchronize()
    assert cache.records == 2 and cache.hits == 2 and cache.eager_steps == 3, (
        cache.records, cache.hits, cache.eager_steps)
    assert l1 == l2, (l1, l2)
    for (k, a), (_, b) in zip(m1.state_dict().items(), m2.state_dict().items()):
        assert torch.equal(a, b), k
