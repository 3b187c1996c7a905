"""Loss of the training step: calc_loss_BCE + 0.8 * calc_loss_L1 (train.py:176-216, :595-597).

The BCE weight is the scalar ratio N*H*W / #(gt >= 0.5) over the WHOLE global batch
(DataParallel gathers outputs to GPU 0 before the loss).  Under DDP each rank holds a shard,
so the positive count is all-reduced before the ratio is formed, which keeps the reference's
global-batch semantics.  The count needs one host sync, exactly like the reference's .item().
"""
import torch
import torch.distributed as dist

from . import functions as fn


def global_ratio(cnt, total, group=None):
    """N*H*W / #(gt >= 0.5) over the global batch: (cnt, total) int64 [1] tensors are
    summed over ranks when a process group is up.  None if there is no positive pixel
    (train.py:185-187 falls back to an unweighted BCE)."""
    if dist.is_available() and dist.is_initialized():
        both = torch.cat([cnt.reshape(1), total.reshape(1)])
        dist.all_reduce(both, group=group)
        cnt, total = both[:1], both[1:]
    npos = int(cnt.item())
    if npos == 0:
        return None
    return float(int(total.item())) / npos


def positive_ratio(label, group=None):
    cnt = fn.count_positive(label)
    n, _, h, w = label.shape
    total = torch.tensor([n * h * w], dtype=torch.int64, device=label.device)
    return global_ratio(cnt, total, group)


def calc_loss_BCE(pred, label, ratio="auto"):
    if ratio == "auto":
        ratio = positive_ratio(label)
    w = 1.0 if ratio is None else ratio
    return fn.BceL1Fn.apply(pred, label, w, 0.0)


def calc_loss_L1(pred, label):
    return fn.BceL1Fn.apply(pred, label, 0.0, 1.0)


def bce_l1(pred, label, ratio="auto", l1_weight=0.8):
    """calc_loss_BCE(pred, label) + l1_weight * calc_loss_L1(pred, label) in one kernel."""
    if ratio == "auto":
        ratio = positive_ratio(label)
    w = 1.0 if ratio is None else ratio
    return fn.BceL1Fn.apply(pred, label, w, l1_weight)


def bce_l1_device(pred, label, l1_weight=0.8, group=None):
    """bce_l1 with the positive count kept on the device (all-reduced asynchronously under
    DDP): no host sync, HIP-graph capturable.  Same value as bce_l1."""
    cnt = fn.count_positive(label)
    n, _, h, w = label.shape
    total = n * h * w
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(cnt, group=group)
        total *= dist.get_world_size(group)
    return fn.BceL1DevFn.apply(pred, label, cnt, total, l1_weight)
