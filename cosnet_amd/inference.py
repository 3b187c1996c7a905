"""N-reference inference of test.py (:287-305) and its evaluation (:307-344).

The reference re-encodes the target frame once per reference frame and averages x1 over the
N forwards.  In eval mode every op is per-sample (BN uses running statistics), so encoding
the target once, the N search frames as one batch, and running the co-attention head on the
N-way stack gives the same average (6e-8 in fp32) with 1 + N instead of 2N
encoder passes.
"""
import torch

from . import _native as nv
from . import ops


@torch.no_grad()
def multi_reference_x1(model, target, target_depth, searches, search_depths):
    """target [1,3,H,W], target_depth [1,1,H,W], searches [N,3,H,W], search_depths [N,1,H,W]
    (fp32 NCHW on the GPU) -> mean over the N references of x1, [1,1,H,W] fp32."""
    if model.training:
        raise RuntimeError("multi-reference inference runs in eval mode (test.py:230)")
    model._set_dtype()
    target, target_depth, searches, search_depths = map(
        model._prep, (target, target_depth, searches, search_depths))
    n = searches.shape[0]
    input_size = tuple(target.shape[2:])
    va, geo1 = model.encoder.features_nhwc(target)
    da, _ = model.depth_encoder.features_nhwc(target_depth)
    vb, geo = model.encoder.features_nhwc(searches)
    db, _ = model.depth_encoder.features_nhwc(search_depths)
    p1 = va.shape[0]
    va_n = torch.empty((n * p1, va.shape[1]), dtype=va.dtype, device=va.device)
    da_n = torch.empty_like(va_n)
    for i in range(n):  # stack the target features N times (one copy kernel each)
        ops.cast_copy(va, va_n[i * p1:(i + 1) * p1])
        ops.cast_copy(da, da_n[i * p1:(i + 1) * p1])
    x1, _ = model.head_nhwc(va_n, vb, da_n, db, geo, input_size)
    out = torch.empty((1, 1) + input_size, dtype=torch.float32, device=x1.device)
    hw = input_size[0] * input_size[1]
    # mean over the N outputs: a fixed-order [N][HW] -> [HW] column reduction scaled by 1/N
    x1 = x1.contiguous()
    nv.call("cn_mean_rows", x1.data_ptr(), n, hw, out.data_ptr(), nv.stream())
    return out


@torch.no_grad()
def resize_linear(x, out_hw):
    """cv2.resize(..., INTER_LINEAR) of a float map (half-pixel centres, no antialias), which is
    bilinear with align_corners=False: the upsample kernel without the sigmoid."""
    n, c, h, w = x.shape
    assert c == 1
    H, W = out_hw
    if (H, W) == (h, w):
        return x
    out = torch.empty((n, 1, H, W), dtype=torch.float32, device=x.device)
    src = x.contiguous()
    nv.call("cn_upsample_sigmoid", src.data_ptr(), n, h, w, H, W, 0, out.data_ptr(), nv.stream())
    return out


def masks_uint8(x):
    """(output * 255).astype(np.uint8) of test.py:317 (truncation toward zero)."""
    return (x.detach().float().cpu().numpy() * 255).astype("uint8")


@torch.no_grad()
def soft_iou(x, gt):
    """GPU quantisation + soft-J of test.py:317 / evaluation.py:3-22 (HIP kernel cn_soft_iou).

    x: [n,1,H,W] (or [n,H,W]) fp32 in [0,1] on the GPU; gt: [n,H,W] {0,1} (any integer / bool /
    float dtype holding 0/1; converted to uint8 like the reference's astype).
    Returns (masks [n,H,W] uint8 on the GPU, iou [n] float64 on the GPU, counts [n,4] int64 =
    (sum p&g, sum p|g, nonzero p, nonzero g)).  Bit-exact with evaluation.compute_iou on the
    host masks."""
    n = x.shape[0]
    hw = x.shape[-2] * x.shape[-1]
    if x.dtype != torch.float32 or not x.is_cuda:
        raise RuntimeError("soft_iou: x must be fp32 on the GPU")
    if gt.shape[0] != n or gt.shape[-2] * gt.shape[-1] != hw:
        raise RuntimeError("soft_iou: gt %s does not match x %s" % (tuple(gt.shape), tuple(x.shape)))
    x = x.contiguous()
    g = gt.to(device=x.device, dtype=torch.uint8).contiguous()
    masks = torch.empty((n,) + tuple(x.shape[-2:]), dtype=torch.uint8, device=x.device)
    iou = torch.empty((n,), dtype=torch.float64, device=x.device)
    counts = torch.empty((n, 4), dtype=torch.int64, device=x.device)
    nv.call("cn_soft_iou", x.data_ptr(), g.data_ptr(), n, hw, masks.data_ptr(), iou.data_ptr(),
            counts.data_ptr(), nv.stream())
    return masks, iou, counts
