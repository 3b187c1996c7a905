"""The data-parallel gradient layout and bucket reduction of TrainStep (train_step.py) on CPU,
world_size 2 over gloo: the arena/bucket plan covers every trainable parameter exactly once,
the two head buckets split the RGB head + decoder from the depth head, every encoder segment has
a bucket of its own holding exactly that segment's parameters in production order, issued from
its encoder's stream, slots are 64-byte aligned, and the per-bucket async all-reduce sums
the ranks' 1/world-scaled buckets into DataParallel's mean.  (The pre-scale and the SGD are
HIP kernels; their GPU coverage is tests/test_gpu_dataparallel.py.)"""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import cosnet_amd as C
        from cosnet_amd.optim import reference_param_groups
        from cosnet_amd.train_step import TrainStep

        torch.manual_seed(0)
        m = C.build_model(torch.float32)
        m.encoder.main_classifier.requires_grad_(False)
        g0, g1 = reference_param_groups(m)
        ts = TrainStep.__new__(TrainStep)        # the planning half only (no device tables)
        ts.model, ts.group, ts.world, ts.grad_dtype = m, None, world, "fp32"
        ts.coll = True     # world > 1 (or world 1 with TrainStep collectives=True)
        seen, ts.params = set(), []
        for p in list(g0) + list(g1):
            if id(p) not in seen:
                seen.add(id(p))
                ts.params.append(p)
        ts._dp_setup()
        dp = ts.dp
        got = [p for b in dp["buckets"] for p in b]
        ok_cover = (len({id(p) for p in got}) == len(got) ==
                    len({id(p) for p in ts.params}))
        ok_align = all(a % 16 == 0 for a, _ in dp["ranges"])
        ok_contig = all(dp["ranges"][i][1] == dp["ranges"][i + 1][0] for i in range(len(dp["ranges"]) - 1))
        ok_alias = all(dp["views"][p].data_ptr() == dp["arena"][p].data_ptr() for p in got)
        ok_stage = len(dp["pieces"]) == 4 + 3
        # bucket 0 = RGB head + decoder, bucket 1 = depth head, then one bucket per encoder
        # segment: depth segment j (depth stream) before RGB segment j (the step's stream)
        dep_head = {id(p) for mod in (m.depth_similarity_weights, m.depth_gate, m.depth_reduce_channels,
                                      m.depth_bn, m.depth_weights) for p in mod.parameters()}
        ok_stage &= {id(p) for p in dp["buckets"][1]} == dep_head
        ok_stage &= not any(id(p) in dep_head for p in dp["buckets"][0])
        for i, (d, k, bk, role) in enumerate(dp["pieces"]):
            want = [p for p in d.segment_params(k) if any(p is q for q in ts.params)]
            ok_stage &= bk == i + 2 and [id(p) for p in dp["buckets"][bk]] == [id(p) for p in want]
            ok_stage &= role == ("s2" if "Depth" in type(d.enc).__name__ else "s1")
        # every rank writes (rank + 1) / world into its buckets (the in-graph 1/world pre-scale),
        # the per-bucket async all-reduce must leave the mean (1 + 2) / 2 everywhere
        dp["flat"].fill_((rank + 1) / world)
        for k in range(len(dp["buckets"])):
            ts._dp_launch_reduce(k)
        for w in dp["works"]:
            w.wait()
        a, b = dp["ranges"][0][0], dp["ranges"][-1][1]
        red = dp["flat"][a:b]
        nb = sum(1 for a_, b_ in dp["ranges"] if b_ > a_)
        ok_stage &= dp["issued"] == nb
        q.put((rank, ok_cover, ok_align, ok_contig, ok_alias, ok_stage, len(dp["pieces"]),
               float(red.min()), float(red.max())))
    finally:
        dist.destroy_process_group()


def _run(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for rank, cover, align, contig, alias, stage, nseg, lo, hi in res:
        assert cover and align and contig and alias and stage, (rank, cover, align, contig, alias, stage)
        assert nseg == 7          # RGB: ASPP+layer4, layer3 x2, layer2+1+stem; depth: 3 of them
        want = sum(r + 1 for r in range(world)) / world
        assert lo == hi == want, (lo, hi)


def test_bucket_plan_and_reduction_two_ranks():
    _run(2)


def test_bucket_reduction_world1_collectives():
    """World 1 with collectives on (bench.py --dp-chain 1 --dist-backend nccl issues the same
    calls on a world-1 RCCL group): every non-empty bucket's all-reduce is really issued."""
    _run(1)


def test_collectives_need_a_process_group():
    import pytest
    import cosnet_amd as C
    from cosnet_amd.optim import SGD, reference_param_groups
    from cosnet_amd.train_step import TrainStep
    if dist.is_initialized():
        pytest.skip("process group present")
    m = C.build_model(torch.float32)
    g0, g1 = reference_param_groups(m)
    with pytest.raises(RuntimeError, match="process group"):
        TrainStep(m, SGD([g0, g1], [0.0, 0.0]), 2, 65, collectives=True)
