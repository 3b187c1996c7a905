"""Name-keyed deterministic weight recipe (SURVEY.md §8c "Golden-vector plan" item 1).

The reference initialises every conv with N(0, 0.01) (rgbd_segmentation_RAA.py:53-62,
deeplab/residual_net.py:116-121, deeplab/deeplabv3_encoder.py:36-42,106-111,163-168).  At
that scale the co-attention softmax is uniform and the model output is a constant 0.5002,
so parity measured there says nothing.  Tests and benchmarks therefore use this recipe:
every state_dict entry is drawn from its own CPU generator seeded by crc32(key), so the
fixture generator (which runs the reference) and the tests (which run this package) get
bit-identical weights without committing 543 MB of tensors.

  conv / linear weight : N(0, 2 / fan_in)          (Kaiming fan_in, keeps BN-free heads sane)
  conv bias            : N(0, 0.01^2)
  BN weight / bias     : 1 + N(0, 0.1^2) / N(0, 0.1^2)
  BN running stats     : mean 0, var 1 (torch defaults; calibrated separately)
  PReLU weight         : 0.25 (torch default)
  num_batches_tracked  : 0
"""
import math
import zlib

import torch


def _gen(key):
    return torch.Generator().manual_seed(zlib.crc32(key.encode("utf-8")))


def recipe_tensor(key, shape, dtype):
    """Deterministic value for one state_dict entry."""
    shape = tuple(shape)
    if key.endswith("num_batches_tracked"):
        return torch.zeros(shape, dtype=dtype)
    if key.endswith("running_mean"):
        return torch.zeros(shape, dtype=dtype)
    if key.endswith("running_var"):
        return torch.ones(shape, dtype=dtype)
    if key.endswith("prelu.weight"):
        return torch.full(shape, 0.25, dtype=dtype)
    g = _gen(key)
    if len(shape) >= 2:  # conv [Cout, Cin, kh, kw] or linear [out, in]
        fan_in = 1
        for s in shape[1:]:
            fan_in *= s
        std = math.sqrt(2.0 / fan_in)
        return (torch.randn(shape, generator=g, dtype=torch.float64) * std).to(dtype)
    # 1-D: BN affine or conv bias
    r = torch.randn(shape, generator=g, dtype=torch.float64)
    is_bn = _is_bn_key(key)
    if is_bn and key.endswith(".weight"):
        return (1.0 + 0.1 * r).to(dtype)
    if is_bn and key.endswith(".bias"):
        return (0.1 * r).to(dtype)
    return (0.01 * r).to(dtype)  # conv bias


def _is_bn_key(key):
    mod = key.rsplit(".", 1)[0]
    last = mod.rsplit(".", 1)[-1]
    if last.startswith("bn") or last in ("depth_bn", "bn_A", "bn_B"):
        return True
    # downsample.1 is the BN of the downsample Sequential (deeplab/residual_net.py:128-131)
    return mod.endswith("downsample.1")


def recipe_state_dict(template):
    """Fill a state_dict-shaped mapping {key: tensor} with recipe values (same dtypes)."""
    out = {}
    for k, v in template.items():
        out[k] = recipe_tensor(k, v.shape, v.dtype)
    return out


BGR_MEAN = (104.00698793, 116.66876762, 122.67891434)  # config.yaml:83


def synthetic_inputs(batch, height, width, seed=1234, correlated=True):
    """Seeded synthetic RGB-D frame pairs.

    rgb = U[0,255) - BGR mean, depth = U[0,255), gt = smooth blobs in {0,1}.
    With correlated=True the counterpart frame is the target rolled by 5 px along W
    (gives a peaked, realistic affinity).  Returns NCHW float32 CPU tensors.
    """
    g = torch.Generator().manual_seed(seed)
    mean = torch.tensor(BGR_MEAN, dtype=torch.float32).view(1, 3, 1, 1)
    rgb_a = torch.rand((batch, 3, height, width), generator=g) * 255.0 - mean
    depth_a = torch.rand((batch, 1, height, width), generator=g) * 255.0
    if correlated:
        rgb_b = torch.roll(rgb_a, 5, -1).contiguous()
        depth_b = torch.roll(depth_a, 5, -1).contiguous()
    else:
        rgb_b = torch.rand((batch, 3, height, width), generator=g) * 255.0 - mean
        depth_b = torch.rand((batch, 1, height, width), generator=g) * 255.0
    gt_a = _blobs(batch, height, width, g)
    gt_b = torch.roll(gt_a, 5, -1).contiguous() if correlated else _blobs(batch, height, width, g)
    return rgb_a, rgb_b, depth_a, depth_b, gt_a, gt_b


def _blobs(batch, height, width, g):
    yy = torch.arange(height, dtype=torch.float32).view(1, height, 1)
    xx = torch.arange(width, dtype=torch.float32).view(1, 1, width)
    out = torch.zeros((batch, 1, height, width))
    for b in range(batch):
        m = torch.zeros((height, width))
        for _ in range(3):
            cy = float(torch.rand((), generator=g)) * height
            cx = float(torch.rand((), generator=g)) * width
            r = (0.1 + 0.2 * float(torch.rand((), generator=g))) * min(height, width)
            m = torch.maximum(m, (((yy - cy) ** 2 + (xx - cx) ** 2) <= r * r).float()[0])
        out[b, 0] = m
    return out
