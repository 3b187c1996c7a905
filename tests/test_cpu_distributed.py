"""Multi-process (gloo, world_size 2) coverage of the data-parallel host logic on CPU."""
import os
import socket

import pytest
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
        from cosnet_amd.loss import global_ratio
        g = torch.Generator().manual_seed(100 + rank)
        gt = (torch.rand((2, 1, 17, 19), generator=g) < (0.2 + 0.2 * rank)).float()
        cnt = torch.tensor([int((gt >= 0.5).sum())], dtype=torch.int64)
        total = torch.tensor([gt.numel()], dtype=torch.int64)
        r = global_ratio(cnt, total)
        # gradient averaging as DDP does it: mean of per-rank grads == global-batch mean
        grad = torch.full((3,), float(rank + 1))
        dist.all_reduce(grad)
        grad /= world
        q.put((rank, r, int(cnt.item()), gt.numel(), grad.tolist()))
    finally:
        dist.destroy_process_group()


def test_global_positive_ratio_matches_dataparallel_semantics():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    res.sort()
    npos = sum(r[2] for r in res)
    tot = sum(r[3] for r in res)
    for r in res:
        # every rank uses the GLOBAL ratio (DataParallel computes the loss on the gathered
        # batch, train.py:183-192), not its shard's
        assert r[1] == pytest.approx(tot / npos, rel=1e-12)
        assert r[4] == [1.5, 1.5, 1.5]


def test_global_ratio_single_process_and_empty():
    from cosnet_amd.loss import global_ratio
    assert global_ratio(torch.tensor([5]), torch.tensor([20])) == 4.0
    assert global_ratio(torch.tensor([0]), torch.tensor([20])) is None
