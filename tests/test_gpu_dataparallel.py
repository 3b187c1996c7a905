"""Data-parallel train step (cosnet_amd.train_step.TrainStep, world > 1) on the GPU.

Two ranks share the box's one MI355X (gloo carries the collectives, RCCL cannot put two ranks
on one device): each rank replays its captured HIP graph on its own frame pairs, the flat
fp32 gradient buffer is averaged across ranks (train.py's DataParallel gradient reduce ->
DDP semantics) and the SGD kernel steps every rank's masters from the SAME
averaged gradient, so the parameters must stay bit-identical across ranks while the ranks'
losses differ.  The BCE positive counts are all-reduced (global-batch weighting).
"""
import os
import socket
import sys

import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir):
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    import torch.distributed as dist
    import cosnet_amd as C
    from cosnet_amd.init_recipe import recipe_state_dict, synthetic_inputs
    from cosnet_amd.optim import SGD, reference_param_groups
    from cosnet_amd.train_step import TrainStep

    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    m = C.build_model(torch.bfloat16)
    m.load_state_dict(recipe_state_dict(m.state_dict()))
    m.encoder.main_classifier.requires_grad_(False)
    m = m.to(dev).train()
    g0, g1 = reference_param_groups(m)
    opt = SGD([g0, g1], [0.0, 0.0])
    step = TrainStep(m, opt, 2, 65, graphed=True)
    step.load(*[t.to(dev) for t in synthetic_inputs(2, 65, 65, seed=100 + rank)])
    lrs = [2.5e-6, 2.5e-3]
    opt.set_lrs(lrs)
    step.capture(warmup=1)          # one eager data-parallel step, then the recorded graph
    losses = [float(step.loss.item())]
    for _ in range(2):
        losses.append(float(step(lrs).item()))
    torch.cuda.synchronize()
    flat = torch.cat([p.detach().float().flatten() for p in m.parameters()])
    summary = torch.tensor([flat.double().sum().item(), flat.double().square().sum().item(),
                            float(step.cnt[0].item()), float(step.cnt[1].item())] + losses,
                           dtype=torch.float64)
    torch.save({"summary": summary, "head": flat[:4096].cpu()},
               os.path.join(outdir, "rank%d.pt" % rank))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_two_rank_graph_step_keeps_ranks_in_sync(cuda, tmp_path):
    import torch.multiprocessing as mp
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    r = [torch.load(os.path.join(str(tmp_path), "rank%d.pt" % i), weights_only=True) for i in range(world)]
    s0, s1 = r[0]["summary"], r[1]["summary"]
    # parameters identical on both ranks after 3 averaged-gradient steps
    assert torch.equal(r[0]["head"], r[1]["head"])
    assert s0[0] == s1[0] and s0[1] == s1[1]
    # global positive counts are the same on both ranks (all-reduced)
    assert s0[2] == s1[2] and s0[3] == s1[3]
    # each rank trained on its own pairs: different losses, all finite
    losses0, losses1 = s0[4:], s1[4:]
    assert torch.isfinite(losses0).all() and torch.isfinite(losses1).all()
    assert not torch.equal(losses0, losses1)


def _mean_grad_worker(rank, world, port, outdir, grad_dtype, graphed):
    """One data-parallel SGD step (eager, or the recorded chain of graphs: forward + head,
    one graph per encoder segment with its bucket's async all-reduce between replays, SGD;
    momentum 0, no weight decay) against the update a
    single process computes from the MEAN of the ranks' own gradients (each rank's gradient of
    its shard's loss with the global positive count, train.py:183-192; DataParallel's reduce)."""
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    import torch.distributed as dist
    import cosnet_amd as C
    from cosnet_amd import functions as fn
    from cosnet_amd.init_recipe import recipe_state_dict, synthetic_inputs
    from cosnet_amd.optim import SGD, reference_param_groups
    from cosnet_amd.train_step import TrainStep

    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda:0")

    def model():
        m = C.build_model(torch.bfloat16)
        m.load_state_dict(recipe_state_dict(m.state_dict()))
        m.encoder.main_classifier.requires_grad_(False)
        return m.to(dev).train()

    ins = [t.to(dev) for t in synthetic_inputs(2, 65, 65, seed=200 + rank)]
    lr = 1e-3
    # reference: this rank's own gradient, global positive counts, then the mean over ranks
    ref = model()
    cnt = torch.stack([fn.count_positive(ins[4])[0], fn.count_positive(ins[5])[0]])
    dist.all_reduce(cnt)
    x1, x2, _ = ref(*ins[:4])
    loss = fn.BceL1PairDevFn.apply(x1, x2, ins[4], ins[5], cnt, 2 * 65 * 65 * world, 0.8)
    loss.backward()
    names = [k for k, p in ref.named_parameters() if p.grad is not None]
    g = torch.cat([dict(ref.named_parameters())[k].grad.float().flatten() for k in names])
    dist.all_reduce(g)
    g /= world
    # the data-parallel step under test
    m = model()
    p0 = torch.cat([dict(m.named_parameters())[k].detach().float().flatten() for k in names])
    g0, g1 = reference_param_groups(m)
    opt = SGD([g0, g1], [lr, lr], momentum=0.0, weight_decay=0.0)
    if graphed:
        # one eager warm-up step at lr 0 (masters unchanged: momentum 0, no weight decay), then
        # record, then ONE replay at lr: the update comes from the graphs alone
        step = TrainStep(m, opt, 2, 65, graphed=True, grad_dtype=grad_dtype)
        step.load(*ins)
        opt.set_lrs([0.0, 0.0])
        step.capture(warmup=1)
        step([lr, lr])
    else:
        step = TrainStep(m, opt, 2, 65, graphed=False, grad_dtype=grad_dtype)
        step.run_batch(*ins, [lr, lr])
    torch.cuda.synchronize()
    p1 = torch.cat([dict(m.named_parameters())[k].detach().float().flatten() for k in names])
    torch.save({"dp": ((p0 - p1) / lr).cpu(), "mean": g.cpu()}, os.path.join(outdir, "mg%d.pt" % rank))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("graphed", [False, True])
@pytest.mark.parametrize("grad_dtype", ["fp32", "bf16"])
def test_two_rank_update_is_mean_of_rank_gradients(cuda, tmp_path, grad_dtype, graphed):
    import torch.multiprocessing as mp
    world = 2
    mp.spawn(_mean_grad_worker, args=(world, _free_port(), str(tmp_path), grad_dtype, graphed),
             nprocs=world,
             join=True)
    for r in range(world):
        d = torch.load(os.path.join(str(tmp_path), "mg%d.pt" % r), weights_only=True)
        got, want = d["dp"].double(), d["mean"].double()
        # p1 = p0 - lr * g in fp32: the recovered g carries the masters' fp32 rounding
        # (|p| / lr * 2^-24); bf16 reduction adds one bf16 rounding of each rank's gradient
        tol = 1e-3 if grad_dtype == "fp32" else 1e-2
        err = ((got - want).abs().max() / want.abs().max()).item()
        assert err <= tol, (r, err)
