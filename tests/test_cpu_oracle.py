"""CPU suite: pins the oracle (oracle/model_ref.py) to the reference's golden fixtures, and
checks the host-side logic of the product package that runs without a GPU.
"""
import os
import re

import numpy as np
import pytest
import torch

from conftest import REPO, golden, golden_meta
from cosnet_amd.init_recipe import recipe_state_dict
from oracle.model_ref import RefModel, compute_iou, loss_bce_l1


def _template():
    import cosnet_amd as C
    torch.manual_seed(0)
    return C.build_model()


@pytest.fixture(scope="module")
def model_cpu():
    return _template()


def test_state_dict_schema_matches_reference(model_cpu):
    meta = golden_meta()["state_dict"]
    sd = model_cpu.state_dict()
    assert [k for k, _, _ in meta] == list(sd.keys())
    for k, shape, dt in meta:
        assert list(sd[k].shape) == shape and str(sd[k].dtype) == dt, k
    assert len(sd) == 1059
    assert sum(p.numel() for p in model_cpu.parameters()) == 142371334


def test_seeded_init_is_bit_identical_to_reference(model_cpu):
    """Same module construction order and init loops => torch.manual_seed(0) gives the
    reference's exact weights (rgbd_segmentation_RAA.py:53-62 and nested inits)."""
    ref = golden_meta()["init_seed0"]
    sd = model_cpu.state_dict()
    for k, (s, a, first) in ref.items():
        v = sd[k].contiguous().double()
        assert float(v.sum()) == s and float(v.abs().sum()) == a and float(v.flatten()[0]) == first, k


def test_param_groups_match_train_py(model_cpu):
    from cosnet_amd.optim import reference_param_groups
    meta = golden_meta()["param_groups"]
    names = {id(p): k for k, p in model_cpu.named_parameters()}
    g0, g1 = reference_param_groups(model_cpu, duplicate_params=True)
    assert [names[id(p)] for p in g0] == meta["group0"]
    assert [names[id(p)] for p in g1] == meta["group1"]
    u0, _ = reference_param_groups(model_cpu, duplicate_params=False)
    assert len(u0) == len(set(meta["group0"]))


def test_load_state_key_remap(model_cpu):
    """load_state strips module. and maps the original-COSNet names (rgbd_segmentation_RAA.py:103-136)."""
    sd = model_cpu.state_dict()
    legacy = {}
    for k, v in sd.items():
        nk = k
        for a, b in (("encoder.aspp.", "encoder.layer5."), ("rgb_similarity_weights.", "linear_e."),
                     ("reduce_channels_A.", "conv1."), ("bn_A.", "bn1."),
                     ("segmentation_classifier_B.", "main_classifier2.")):
            if nk.startswith(a):
                nk = b + nk[len(a):]
        if nk.startswith("encoder.backbone."):
            nk = "encoder." + nk[len("encoder.backbone."):]
        legacy["module." + nk] = v.clone() + (1 if v.is_floating_point() else 0)
    import cosnet_amd as C
    m = C.build_model()
    m.load_state(legacy)
    sd2 = m.state_dict()
    for k in sd:
        if sd[k].is_floating_point():
            assert torch.equal(sd2[k], sd[k] + 1), k


def _oracle(dtype, bn_calib=None):
    tmpl = _template().state_dict()
    sd = recipe_state_dict(tmpl)
    if bn_calib is not None:
        for k in bn_calib.files:
            sd[k[len("calib/"):]] = torch.from_numpy(bn_calib[k])
    return RefModel(sd, dtype=dtype)


def test_oracle_train_step_matches_reference_fp64():
    z = golden("train_b2_97.npz")
    meta = golden_meta()["train_b2_97"]
    ref = _oracle(torch.float64)
    inp = [torch.from_numpy(z["in/" + k]).double() for k in
           ("rgb_a", "rgb_b", "depth_a", "depth_b", "gt_a", "gt_b")]
    st = {}
    x1, x2, labels = ref.forward(*inp[:4], stages=st)
    loss = loss_bce_l1(x1, inp[4]) + loss_bce_l1(x2, inp[5])
    loss.backward()
    for name, t in (("x1", x1), ("x2", x2), ("labels", labels), ("loss", loss.reshape(1))):
        assert np.abs(t.detach().numpy() - z["f64/" + name]).max() <= 1e-9, name
    norms = np.array([ref.p[k].grad.norm().item() for k in meta["grad_norm_keys"]])
    r = z["f64/grad_norm"]
    assert (np.abs(norms - r) <= 1e-8 * np.maximum(r, 1e-3)).all()
    for k in ["encoder.backbone.bn1.running_mean", "bn_A.running_mean", "depth_bn.running_mean"]:
        assert np.abs(ref.p[k].numpy() - z["f64/buf/" + k]).max() <= 1e-10, k


@pytest.mark.parametrize("tag", ["eval_b1_97"])
def test_oracle_eval_matches_reference_fp64(tag):
    z = golden(tag + ".npz")
    ref = _oracle(torch.float64, golden("bn_calibration.npz"))
    ref.training = False
    inp = [torch.from_numpy(z["in/" + k]).double() for k in ("rgb_a", "rgb_b", "depth_a", "depth_b")]
    with torch.no_grad():
        x1, x2, labels = ref.forward(*inp)
    # same (fp32-committed) BN calibration on both sides: fp64 agreement
    for name, t in (("x1", x1), ("x2", x2), ("labels", labels)):
        assert np.abs(t.numpy() - z["f64/" + name]).max() <= 1e-9, name


def test_compute_iou_known_answers():
    from cosnet_amd.evaluation import compute_iou as product_iou
    for case in golden_meta()["compute_iou"]:
        pred = np.array(case["pred"], dtype=np.uint8)
        gt = np.array(case["gt"], dtype=np.uint8)
        assert compute_iou(pred, gt) == pytest.approx(case["iou"], abs=0, rel=1e-15)
        assert product_iou(pred, gt) == pytest.approx(case["iou"], abs=0, rel=1e-15)


def test_lr_poly_matches_train_py():
    from cosnet_amd.optim import lr_poly
    assert lr_poly(2.5e-4, 0, 100, 0.9, 0) == 2.5e-4
    assert lr_poly(2.5e-4, 50, 100, 0.9, 7) == pytest.approx(2.5e-4 * 0.5 * 0.5 ** 0.9)


def test_library_exports_every_header_symbol():
    """The C ABI library loads (no GPU needed) and exports every symbol include/*.h declares."""
    import ctypes
    from cosnet_amd import _native
    if not os.path.exists(_native.LIB_PATH):
        import __graft_entry__
        __graft_entry__.build()
    lib = ctypes.CDLL(_native.LIB_PATH)
    hdr = open(os.path.join(REPO, "include", "cosnet_hip.h")).read()
    names = set(re.findall(r"^(?:int|size_t|const char\*)\s+(cn_\w+)\(", hdr, re.M))
    assert len(names) >= 30
    for n in sorted(names):
        assert hasattr(lib, n), n
    assert names == set(_native.exported_symbols())


def test_library_built_from_this_tree():
    """Build provenance: the source hash stamped into the library equals the hash of the HIP
    sources in this tree (a stale .so fails here; build() rebuilds it)."""
    from cosnet_amd import _native
    info = _native.build_info()
    assert info["built_from_tree"], info


def test_forward_requires_gpu_no_cpu_fallback(model_cpu):
    x = torch.zeros(2, 3, 33, 33)
    d = torch.zeros(2, 1, 33, 33)
    with pytest.raises(RuntimeError):
        model_cpu(x, x, d, d)
