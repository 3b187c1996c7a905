"""Parity at the BASELINE configurations themselves (round-2 additions):

* configs[3]: N-reference inference, one target + 5 references at 473x473, against the
  reference's own test.py loop (tests/golden/nref5_473.npz, produced by make_golden.py nref
  from the reference in fp32 / fp64 / bf16) -- fp32 through the materialised path, bf16
  through the fused co-attention kernel (asserted);
* the co-attention block (CoattFn fwd + bwd) at HW = 3600 (60 x 60), B = 4, the training shape
  of configs[1], against the oracle's restatement of rgbd_segmentation_RAA.py:150-170 in fp64;
* configs[1] itself: 473 x 473, B = 4 pairs, bf16, fwd + bwd, and the graphed train step.

Tolerance policy as tests/test_gpu_model.py: fp32 within 8x the reference's own fp32-vs-fp64
floor (stored in the fixture); bf16 at J level, measured against the reference run in bf16.
"""
import zlib

import numpy as np
import pytest
import torch

from conftest import golden
import cosnet_amd as C
from cosnet_amd import loss as L
from cosnet_amd import ops
from cosnet_amd.init_recipe import recipe_state_dict, synthetic_inputs

pytestmark = pytest.mark.gpu


def make_model(cuda, dtype, calib=None):
    m = C.build_model(dtype)
    sd = recipe_state_dict(m.state_dict())
    if calib is not None:
        for k in calib.files:
            sd[k[len("calib/"):]] = torch.from_numpy(calib[k])
    m.load_state_dict(sd)
    return m.to(cuda)


def _nref_inputs(z):
    ra, rb, da, db, _, _ = synthetic_inputs(5, 473, 473, seed=5)
    crc = [zlib.crc32(t.numpy().tobytes()) for t in (ra, rb, da, db)]
    assert crc == list(z["in_crc32"]), "synthetic input generator drifted"
    return ra[:1], da[:1], rb, db


def test_nref5_473_fp32_matches_reference(cuda):
    """configs[3] in fp32: multi_reference_x1 (target encoded once, 5-way stack, sequential-order
    mean / 5) against the reference's loop mean (test.py:287-305) in fp64."""
    from cosnet_amd.inference import multi_reference_x1
    z = golden("nref5_473.npz")
    t, td, rb, db = _nref_inputs(z)
    m = make_model(cuda, torch.float32, golden("bn_calibration_473.npz")).eval()
    got = multi_reference_x1(m, t.to(cuda), td.to(cuda), rb.to(cuda), db.to(cuda))
    torch.cuda.synchronize()
    g = got.double().cpu().numpy().reshape(z["f64r/x1mean"].shape)
    ref = z["f64r/x1mean"].astype(np.float64)
    floor = float(z["floor/x1mean"][0])
    tol = 8 * floor + 1e-5
    err = float(np.abs(g - ref).max())
    assert err <= tol, (err, tol, floor)
    amb = np.abs(ref - 0.5) <= tol
    flips = ((g > 0.5) != (ref > 0.5)) & ~amb
    assert not flips.any(), int(flips.sum())


def test_nref5_473_bf16_fused_in_pipeline(cuda, monkeypatch):
    """configs[3] in bf16: both modalities' co-attention go through the fused kernel (S never in
    HBM), asserted, and the pipeline output equals the same bf16 pipeline with the materialised
    co-attention (affinity GEMM + softmax kernels + gathers) within bf16 rounding of P.

    Why not the fp64 fixture directly: with these random-init weights the 101-layer encoder is
    chaotic in bf16 -- measured at 473x473 eval, V_a of the bf16 HIP model differs from the fp32
    HIP model by 87 % (mean |d| / mean |x|), so bf16 end-to-end outputs are decorrelated from
    fp64 (the reference's own bf16 run decorrelates likewise; its fixture agreement is an
    artefact of saturation).  The bf16 co-attention kernel itself is pinned against fp64 at
    5 x 3600 in tests/test_gpu_coatt_fused.py; the fp32 pipeline against the reference's loop
    mean in the test above."""
    from cosnet_amd.inference import multi_reference_x1
    z = golden("nref5_473.npz")
    t, td, rb, db = _nref_inputs(z)
    m = make_model(cuda, torch.bfloat16, golden("bn_calibration_473.npz")).eval()
    calls = []
    real = ops.coatt_fused
    monkeypatch.setattr(ops, "coatt_fused", lambda *a, **k: calls.append(a[3]) or real(*a, **k))
    args = (t.to(cuda), td.to(cuda), rb.to(cuda), db.to(cuda))
    fused = multi_reference_x1(m, *args)
    assert calls == [5, 5], calls   # RGB and depth co-attention, 5 pairs each
    monkeypatch.setattr(ops, "COATT_FUSED", False)
    mat = multi_reference_x1(m, *args)
    torch.cuda.synchronize()
    assert calls == [5, 5]
    f, g = fused.double().cpu(), mat.double().cpu()
    assert torch.isfinite(f).all() and f.min() >= 0 and f.max() <= 1
    agree = ((f > 0.5) == (g > 0.5)).double().mean().item()
    mad = (f - g).abs().mean().item()
    assert agree >= 0.999 and mad <= 1e-2, (agree, mad)


def test_coattfn_parameter_weight_no_grad_is_fused(cuda, monkeypatch):
    """The model passes its similarity weight as an nn.Parameter (requires_grad=True); under
    torch.no_grad the fused kernel must still be taken."""
    from cosnet_amd.functions import CoattFn
    n, hw, c = 2, 400, 256
    g = torch.Generator().manual_seed(1)
    va = (torch.randn((n * hw, c), generator=g) * 0.7).to(torch.bfloat16).to(cuda)
    vb = (torch.randn((n * hw, c), generator=g) * 0.7).to(torch.bfloat16).to(cuda)
    W = torch.nn.Parameter((torch.randn((c, c), generator=g) * c ** -0.5).to(cuda))
    calls = []
    real = ops.coatt_fused
    monkeypatch.setattr(ops, "coatt_fused", lambda *a, **k: calls.append(1) or real(*a, **k))
    with torch.no_grad():
        CoattFn.apply(va, vb, W, (n, hw))
    assert calls == [1]
    va.requires_grad_(True)
    za, zb = CoattFn.apply(va, vb, W, (n, hw))   # grad mode: training path, not the fused one
    assert calls == [1] and za.requires_grad


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_coattention_block_hw3600_b4(cuda, dt):
    """CoattFn forward AND backward at the configs[1] training shape (B = 4 pairs, 60 x 60
    features, C = 256, S of 3600 x 3600 per pair) against the oracle in fp64 (computed on the
    device: test arithmetic, not the product path).  Logits std ~16 as in the model.
    fp32 2e-4 of the output scale; bf16 0.15 (P and V_a W^T rounded to bf16, SURVEY §7 iii)."""
    from oracle.model_ref import RefModel
    from cosnet_amd.functions import CoattFn
    n, c, h, w = 4, 256, 60, 60
    gen = torch.Generator().manual_seed(36)

    def rnd(shape, scale=1.0):
        return (torch.randn(shape, generator=gen, dtype=torch.float64) * scale).to(dt).double()

    va, vb = rnd((n, c, h, w)), rnd((n, c, h, w))
    W = rnd((c, c), c ** -0.5).float().double()
    gza, gzb = rnd((n, c, h, w)), rnd((n, c, h, w))
    var = va.to(cuda).requires_grad_(True)
    wr = W.to(cuda).requires_grad_(True)
    za, zb = RefModel.coattention(None, var, vb.to(cuda), wr)
    ((za * gza.to(cuda)).sum() + (zb * gzb.to(cuda)).sum()).backward()
    nhwc = lambda x: x.permute(0, 2, 3, 1).reshape(n * h * w, c)
    vag = nhwc(va).to(dt).to(cuda).contiguous().requires_grad_(True)
    vbg = nhwc(vb).to(dt).to(cuda).contiguous()
    Wg = W.float().to(cuda).requires_grad_(True)
    ga, gb = CoattFn.apply(vag, vbg, Wg, (n, h * w))
    torch.autograd.backward([ga, gb], [nhwc(gza).to(dt).to(cuda), nhwc(gzb).to(dt).to(cuda)])
    torch.cuda.synchronize()
    tol = {torch.float32: 2e-4, torch.bfloat16: 0.15}[dt]
    nchw = lambda t: t.reshape(n, h, w, c).permute(0, 3, 1, 2)
    for name, got, ref in (("Z_a", nchw(ga), za), ("Z_b", nchw(gb), zb),
                           ("dV_a", nchw(vag.grad), var.grad), ("dW", Wg.grad, wr.grad)):
        got, ref = got.double(), ref.detach().double()
        err = ((got - ref).abs().max() / ref.abs().max()).item()
        assert err <= tol, (name, err, tol)


def _step_once(m, inp):
    x1, x2, _ = m(*inp[:4])
    loss = L.bce_l1(x1, inp[4]) + L.bce_l1(x2, inp[5])
    return x1, x2, loss


def _grad_norms(m):
    return np.array([p.grad.double().norm().item() for p in m.parameters() if p.grad is not None])


def test_configs1_473_b4_bf16_step_tracks_fp32(cuda):
    """configs[1]: 473 x 473, 4 frame pairs, bf16, fwd + loss + bwd on the HIP path, with the
    same inputs / weights through the fp32 HIP path as the yardstick (the oracle cannot run this
    size in a test's time budget; the fp32 path itself is pinned to the reference fixtures).
    The random-init 101-layer network is chaotic in bf16 (pixel masks decorrelate: measured 85 %
    agreement with fp32 outside |x - 0.5| <= 0.05), so the comparison is on the aggregates a
    training step consumes: finite loss and gradients; |loss_bf16 - loss_fp32| <= 3 % of
    loss_fp32; mean(x1), mean(x2) within 0.03; per-parameter gradient norms: median ratio to
    fp32 within [0.8, 1.25] and >= 90 % of the parameters within [0.5, 2] (single tensors,
    e.g. early BN affines, swing with the chaotic trajectory)."""
    inp = [t.to(cuda) for t in synthetic_inputs(4, 473, 473, seed=1234)]
    m32 = make_model(cuda, torch.float32).train()
    r1, r2, rloss = _step_once(m32, inp)
    rloss.backward()
    torch.cuda.synchronize()
    ref = (rloss.item(), r1.mean().item(), r2.mean().item(), _grad_norms(m32))
    del m32, r1, r2, rloss
    torch.cuda.empty_cache()
    m = make_model(cuda, torch.bfloat16).train()
    x1, x2, loss = _step_once(m, inp)
    loss.backward()
    torch.cuda.synchronize()
    assert np.isfinite(loss.item())
    for p in m.parameters():
        if p.grad is not None:
            assert torch.isfinite(p.grad).all()
    got = (loss.item(), x1.mean().item(), x2.mean().item(), _grad_norms(m))
    assert abs(got[0] - ref[0]) <= 0.03 * abs(ref[0]), (got[:3], ref[:3])
    assert abs(got[1] - ref[1]) <= 0.03 and abs(got[2] - ref[2]) <= 0.03, (got[:3], ref[:3])
    ratio = got[3] / np.maximum(ref[3], 1e-30)
    inside = ((ratio >= 0.5) & (ratio <= 2.0)).mean()
    assert 0.8 <= np.median(ratio) <= 1.25 and inside >= 0.9, (np.median(ratio), inside)


def test_configs1_graphed_train_step_bf16(cuda):
    """configs[1] through the recorded HIP-graph step bench.py times: two replays after the
    eager warmup give finite losses and finite, changed parameters."""
    from cosnet_amd.optim import SGD, reference_param_groups
    from cosnet_amd.train_step import TrainStep
    m = make_model(cuda, torch.bfloat16).train()
    m.encoder.main_classifier.requires_grad_(False)
    g0, g1 = reference_param_groups(m)
    opt = SGD([g0, g1], [2.5e-6, 2.5e-3], momentum=0.9, weight_decay=5e-4)
    step = TrainStep(m, opt, 4, 473)
    step.load(*[t.to(cuda) for t in synthetic_inputs(4, 473, 473, seed=1234)])
    step.capture(warmup=1)
    w0 = m.reduce_channels_A.weight.detach().clone()
    losses = [step([2.5e-6, 2.5e-3]).item() for _ in range(2)]
    torch.cuda.synchronize()
    assert all(np.isfinite(losses)), losses
    assert not torch.equal(w0, m.reduce_channels_A.weight.detach())
    for p in m.parameters():
        assert torch.isfinite(p).all()
