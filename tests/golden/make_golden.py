"""Generate the golden fixtures under tests/golden/ by running the REFERENCE itself.

Run in the build container only (it imports /root/reference, which never ships):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [nref | train473]

Weights come from cosnet_amd.init_recipe (name-keyed, deterministic), inputs from
cosnet_amd.init_recipe.synthetic_inputs (seeded).  Every fixture also carries the same
computation in fp64 so tests can state tolerances relative to the reference's own
fp32-vs-fp64 noise floor (SURVEY.md §8c "Measured noise floors").
"""
import json
import os
import sys
import zlib

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)
sys.path.insert(0, REF)

from cosnet_amd.init_recipe import recipe_state_dict, synthetic_inputs  # noqa: E402

import warnings  # noqa: E402
warnings.filterwarnings("ignore")

from rgbd_segmentation_RAA import RGBDSegmentation_RAA  # noqa: E402  (reference)
from deeplab.residual_net import Bottleneck  # noqa: E402  (reference)
import evaluation  # noqa: E402  (reference)

SELECT = [
    "rgb_similarity_weights.weight", "depth_similarity_weights.weight", "gate.weight",
    "depth_gate.weight", "depth_gate.bias", "bn_A.weight", "bn_A.bias", "depth_bn.weight",
    "depth_weights.bias", "segmentation_classifier_A.weight", "segmentation_classifier_A.bias",
    "segmentation_classifier_B.weight", "encoder.aspp.prelu.weight",
    "encoder.backbone.conv1.weight", "depth_encoder.backbone.conv1.weight",
    "encoder.aspp.bn.weight", "depth_encoder.aspp.conv.bias",
    "encoder.backbone.layer4.2.bn3.weight",
]
HEAD = 2048


def build(dtype):
    torch.manual_seed(0)
    m = RGBDSegmentation_RAA(Bottleneck, [3, 4, 23, 3], [3, 4, 6, 3], num_classes=1)
    sd = recipe_state_dict(m.state_dict())
    m.load_state_dict(sd)
    return m.to(dtype)


def capture(model):
    """Forward hooks that record encoder / depth-encoder outputs (a-side first)."""
    rec = {"enc": [], "denc": []}
    model.encoder.register_forward_hook(lambda mod, i, o: rec["enc"].append(o[0].detach().clone()))
    model.depth_encoder.register_forward_hook(lambda mod, i, o: rec["denc"].append(o.detach().clone()))
    return rec


def loss_fn(pred, gt):
    # restatement of train.py:176-216 (the reference's version calls .cuda())
    npos = int((gt >= 0.5).sum())
    if npos == 0:
        bce = torch.nn.BCELoss()(pred, gt)
    else:
        ratio = gt.shape[0] * gt.shape[2] * gt.shape[3] / npos
        bce = torch.nn.BCELoss(weight=torch.full_like(gt, ratio))(pred, gt)
    return bce + 0.8 * torch.nn.L1Loss()(pred, gt)


def run_train(dtype, inputs):
    m = build(dtype)
    m.train()
    rec = capture(m)
    ra, rb, da, db, ga, gb = [t.to(dtype) for t in inputs]
    x1, x2, labels = m(ra, rb, da, db)
    loss = loss_fn(x1, ga) + loss_fn(x2, gb)
    loss.backward()
    out = {"x1": x1, "x2": x2, "labels": labels, "loss": loss.reshape(1),
           "V_a": rec["enc"][0], "V_b": rec["enc"][1], "D_a": rec["denc"][0],
           "D_b": rec["denc"][1]}
    out = {k: v.detach().double().numpy() for k, v in out.items()}
    named = dict(m.named_parameters())
    gnorm_keys = [k for k, p in named.items() if p.grad is not None]
    out["grad_norm"] = np.array([named[k].grad.double().norm().item() for k in gnorm_keys])
    for k in SELECT:
        g = named[k].grad.detach().double().flatten()
        out["grad_head/" + k] = g[:HEAD].numpy()
        out["grad_nrm/" + k] = np.array([g.norm().item()])
    sd = m.state_dict()
    for k in ["encoder.backbone.bn1.running_mean", "encoder.backbone.bn1.running_var",
              "bn_A.running_mean", "bn_B.running_var", "depth_bn.running_mean",
              "encoder.aspp.bn_x.running_var", "encoder.backbone.bn1.num_batches_tracked",
              "depth_bn.num_batches_tracked"]:
        out["buf/" + k] = sd[k].double().numpy()
    return out, gnorm_keys


def calibrate(dtype, inputs):
    """Eval-mode BN running stats: one train-mode no_grad forward with momentum 1.0."""
    m = build(dtype)
    for mod in m.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            mod.momentum = 1.0
    m.train()
    ra, rb, da, db = [t.to(dtype) for t in inputs[:4]]
    with torch.no_grad():
        m(ra, rb, da, db)
    return {k: v.clone() for k, v in m.state_dict().items()
            if k.endswith("running_mean") or k.endswith("running_var")}


def run_eval(dtype, calib, inputs):
    m = build(dtype)
    sd = m.state_dict()
    for k, v in calib.items():
        sd[k] = v.to(dtype)
    m.load_state_dict(sd)
    m.eval()
    rec = capture(m)
    ra, rb, da, db = [t.to(dtype) for t in inputs[:4]]
    with torch.no_grad():
        x1, x2, labels = m(ra, rb, da, db)
    out = {"x1": x1, "x2": x2, "labels": labels, "V_a": rec["enc"][0], "D_a": rec["denc"][0]}
    return {k: v.double().numpy() for k, v in out.items()}


def put(arr, k, v32, v64):
    """fp32 result, its max-abs distance from fp64 (the noise floor), fp64 for small ones."""
    arr["f32/" + k] = v32
    arr["floor/" + k] = np.array([np.abs(v32 - v64).max()])
    if v64.size <= 4096 or k.startswith("grad") or k in ("x1", "x2", "labels"):
        arr["f64/" + k] = v64


def save(name, arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **{k: (v.astype(np.float32) if v.dtype == np.float64 and
                                     not k.startswith("f64/") else v) for k, v in arrays.items()})
    print("wrote", path, os.path.getsize(path) // 1024, "KiB")


def nref_loop(dtype, calib, target, target_depth, searches, search_depths):
    """test.py:287-305 in eval mode: for each reference i, x1 of model(target, search_i,
    target_depth, search_i_depth) accumulated in an fp32 numpy sum (the reference's
    `output_sum += output[0].cpu().numpy()`), then divided by sample_range."""
    m = build(dtype)
    sd = m.state_dict()
    for k, v in calib.items():
        sd[k] = v.to(dtype)
    m.load_state_dict(sd)
    m.eval()
    n = searches.shape[0]
    out_sum = 0
    with torch.no_grad():
        for i in range(n):
            x1, _, _ = m(target.to(dtype), searches[i:i + 1].to(dtype), target_depth.to(dtype),
                         search_depths[i:i + 1].to(dtype))
            o = x1[0].float().numpy() if dtype != torch.float64 else x1[0].numpy()
            out_sum = out_sum + o
    return out_sum / n


def make_nref():
    """BASELINE configs[3]: one target + 5 references at 473x473, eval mode, with BN running
    statistics calibrated at 473x473 (a 97x97 calibration saturates the 473x473 output: x1 > 0.99
    almost everywhere, which would make the fixture uninformative)."""
    n, size = 5, 473
    calib = calibrate(torch.float64, synthetic_inputs(2, size, size, seed=4321))
    calib = {k: v.float().double() for k, v in calib.items()}
    np.savez_compressed(os.path.join(HERE, "bn_calibration_473.npz"),
                        **{"calib/" + k: v.float().numpy() for k, v in calib.items()})
    ra, rb, da, db, _, _ = synthetic_inputs(n, size, size, seed=5)
    tgt, tdep = ra[:1], da[:1]
    arr = {"in_crc32": np.array([zlib.crc32(t.numpy().tobytes()) for t in (ra, rb, da, db)],
                                dtype=np.int64)}
    f32 = nref_loop(torch.float32, calib, tgt, tdep, rb, db)
    f64 = nref_loop(torch.float64, calib, tgt, tdep, rb, db)
    arr["f32/x1mean"] = f32.astype(np.float32)
    arr["f64r/x1mean"] = f64.astype(np.float32)   # fp64 result rounded to fp32 for storage
    arr["floor/x1mean"] = np.array([np.abs(f32.astype(np.float64) - f64).max()])
    b16 = nref_loop(torch.bfloat16, calib, tgt, tdep, rb, db)
    arr["bf16/x1mean"] = b16.astype(np.float32)
    np.savez_compressed(os.path.join(HERE, "nref5_473.npz"), **arr)
    print("wrote nref5_473.npz", os.path.getsize(os.path.join(HERE, "nref5_473.npz")) // 1024, "KiB")


def make_train473():
    """BASELINE configs[1] pinned to the reference itself: one train step (forward of both
    frames x both modalities, loss, backward) at 473x473 with 4 frame pairs, in fp32 and fp64
    (rgbd_segmentation_RAA.py:139-268, train.py:595-599).  The inputs are the bench's own
    (synthetic_inputs(4, 473, 473, seed=1234), pinned by CRC); outputs are stored on a
    stride-2 pixel grid (the noise floors are over the full tensors), encoder features on a
    channel / pixel subgrid, every parameter's gradient norm, the SELECT gradient heads and
    BN buffers after the step."""
    n, size = 4, 473
    inp = synthetic_inputs(n, size, size, seed=1234)
    f32, gkeys = run_train(torch.float32, inp)
    f64, _ = run_train(torch.float64, inp)
    arr = {"in_crc32": np.array([zlib.crc32(t.numpy().tobytes()) for t in inp], dtype=np.int64)}
    sub = {"x1": (slice(None), slice(None), slice(None, None, 2), slice(None, None, 2)),
           "x2": (slice(None), slice(None), slice(None, None, 2), slice(None, None, 2)),
           "labels": (slice(None), slice(None), slice(None, None, 2), slice(None, None, 2)),
           "V_a": (slice(None), slice(None, None, 8), slice(None, None, 3), slice(None, None, 3)),
           "D_a": (slice(None), slice(None, None, 8), slice(None, None, 3), slice(None, None, 3))}
    for k, v in f32.items():
        if k in ("V_b", "D_b"):
            continue
        if k in sub:
            arr["floor/" + k] = np.array([np.abs(v - f64[k]).max()])
            arr["f32/" + k] = v[sub[k]]
            arr["f64r/" + k] = f64[k][sub[k]]     # fp64 result, stored rounded to fp32
            arr["f64/mean/" + k] = np.array([f64[k].mean()])
            continue
        put(arr, k, v, f64[k])
    save("train_b4_473.npz", arr)
    meta_p = os.path.join(HERE, "meta.json")
    with open(meta_p) as f:
        meta = json.load(f)
    meta["train_b4_473"] = {"grad_norm_keys": gkeys, "select": SELECT, "subgrid": {
        "x1": "[:, :, ::2, ::2]", "V_a": "[:, ::8, ::3, ::3]"}}
    with open(meta_p, "w") as f:
        json.dump(meta, f)
    print("updated meta.json")


def main():
    torch.set_num_threads(os.cpu_count())
    if len(sys.argv) > 1 and sys.argv[1] == "nref":
        make_nref()
        return
    if len(sys.argv) > 1 and sys.argv[1] == "train473":
        make_train473()
        return
    meta = {}
    # ---- 1. train step, B=2, 97x97 -----------------------------------------------------
    inp = synthetic_inputs(2, 97, 97, seed=1234)
    f32, gkeys = run_train(torch.float32, inp)
    f64, _ = run_train(torch.float64, inp)
    arr = {"in/" + n: t.numpy() for n, t in zip(["rgb_a", "rgb_b", "depth_a", "depth_b", "gt_a", "gt_b"], inp)}
    for k, v in f32.items():
        if k in ("V_b", "D_b"):
            continue
        put(arr, k, v, f64[k])
    # the reference run entirely in bf16 (CPU): the bf16 noise floor for J-level parity
    b16, _ = run_train(torch.bfloat16, inp)
    for k in ("x1", "x2", "loss"):
        arr["bf16/" + k] = b16[k].astype(np.float32)
    save("train_b2_97.npz", arr)
    meta["train_b2_97"] = {"grad_norm_keys": gkeys, "select": SELECT}

    # ---- 2. eval forward with calibrated BN stats --------------------------------------
    calib_in = synthetic_inputs(2, 97, 97, seed=4321)
    calib = calibrate(torch.float64, calib_in)
    calib = {k: v.float().double() for k, v in calib.items()}  # what gets committed (fp32)
    arr = {"calib/" + k: v.float().numpy() for k, v in calib.items()}
    save("bn_calibration.npz", arr)
    for (h, w, tag) in [(97, 97, "eval_b1_97"), (240, 320, "eval_b1_240x320")]:
        inp = synthetic_inputs(1, h, w, seed=77)
        e32 = run_eval(torch.float32, calib, inp)
        e64 = run_eval(torch.float64, calib, inp)
        arr = {}
        if h * w <= 97 * 97:
            arr.update({"in/" + n: t.numpy() for n, t in zip(["rgb_a", "rgb_b", "depth_a", "depth_b"], inp)})
        else:
            arr["in_crc32"] = np.array([zlib.crc32(t.numpy().tobytes()) for t in inp[:4]], dtype=np.int64)
        for k in e32:
            if h * w > 97 * 97 and k in ("V_a", "D_a"):
                arr["floor/" + k] = np.array([np.abs(e32[k] - e64[k]).max()])
                continue
            put(arr, k, e32[k], e64[k])
        save(tag + ".npz", arr)

    # ---- 3. SGD param groups of the reference (train.py:220-303 semantics) -------------
    m = build(torch.float32)
    names = {id(p): k for k, p in m.named_parameters()}
    g0 = []
    for mod in m.get_params("encoder"):
        for sub in mod.modules():
            for p in sub.parameters():
                if p.requires_grad:
                    g0.append(names[id(p)])
    g1 = []
    for sub in ("rgb_attention", "depth", "decoder"):
        for mod in m.get_params(sub):
            for p in mod.parameters():
                g1.append(names[id(p)])
    meta["param_groups"] = {"group0": g0, "group1": g1}
    # ---- 3b. state_dict schema and the seeded reference init (torch.manual_seed(0)) ------
    torch.manual_seed(0)
    r = RGBDSegmentation_RAA(Bottleneck, [3, 4, 23, 3], [3, 4, 6, 3], num_classes=1)
    sd = r.state_dict()
    meta["state_dict"] = [[k, list(v.shape), str(v.dtype)] for k, v in sd.items()]
    meta["init_seed0"] = {k: [float(v.double().sum()), float(v.double().abs().sum()),
                              float(v.flatten()[0])] for k, v in sd.items()}

    # ---- 4. compute_iou known answers (evaluation.py:3-22) -----------------------------
    rng = np.random.RandomState(5)
    cases = []
    for i in range(6):
        pred = (rng.rand(24, 32) * 255).astype(np.uint8)
        if i == 0:
            gt = np.zeros((24, 32), np.uint8)
        elif i == 1:
            gt = np.ones((24, 32), np.uint8)
        else:
            gt = (rng.rand(24, 32) < 0.3).astype(np.uint8)
        if i == 2:
            pred[:] = 0
        cases.append({"pred": pred.tolist(), "gt": gt.tolist(),
                      "iou": float(evaluation.compute_iou(pred, gt))})
    meta["compute_iou"] = cases
    with open(os.path.join(HERE, "meta.json"), "w") as f:
        json.dump(meta, f)
    print("wrote meta.json")
    make_nref()


if __name__ == "__main__":
    main()
