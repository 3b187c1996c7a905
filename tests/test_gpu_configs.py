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


class _RoundBF16(torch.autograd.Function):
    """bf16 storage point of the HIP path: rounds the value and the gradient through it."""

    @staticmethod
    def forward(ctx, x):
        return x.to(torch.bfloat16).double()

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.bfloat16).double()


def _coatt_ref(va, vb, w, emul):
    """rgbd_segmentation_RAA.py:150-170 in fp64 (oracle.model_ref.RefModel.coattention's op
    sequence); emul=True rounds V_a W^T to bf16 where the bf16 HIP path stores it."""
    import torch.nn.functional as Fn
    n, c, h, wd = va.shape
    va_f, vb_f = va.reshape(n, c, h * wd), vb.reshape(n, c, h * wd)
    va_t = Fn.linear(va_f.transpose(1, 2), w)
    if emul:
        va_t = _RoundBF16.apply(va_t)
    s = torch.bmm(va_t, vb_f)
    z_b = torch.bmm(va_f, Fn.softmax(s, dim=1))
    z_a = torch.bmm(vb_f, Fn.softmax(s.transpose(1, 2), dim=1))
    return z_a.reshape(n, c, h, wd), z_b.reshape(n, c, h, wd)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_coattention_block_hw3600_b4(cuda, dt):
    """CoattFn forward AND backward at the configs[1] training shape (B = 4 pairs, 60 x 60
    features, C = 256, S of 3600 x 3600 per pair) against the reference op sequence in fp64
    (computed on the device: test arithmetic, not the product path).  Logits std ~16 as in the
    model.  fp32: 2e-4 of the output scale.  bf16: 3e-2 of the output scale (the bound the flash
    kernels meet in tests/test_gpu_coatt_fused.py) against fp64 with V_a W^T rounded to bf16
    where the HIP path stores it, and no further from pure fp64 than that rounding itself puts
    it (<= 1.25 x its own distance + 2e-3): at logits of std 16 one bf16 rounding of V_a W^T moves
    S by ~0.05, i.e. P by ~5 %, for ANY bf16 implementation (measured 3.3e-2 vs pure fp64)."""
    from cosnet_amd.functions import CoattFn
    n, c, h, w = 4, 256, 60, 60
    gen = torch.Generator().manual_seed(36)

    def rnd(shape, scale=1.0):
        return (torch.randn(shape, generator=gen, dtype=torch.float64) * scale).to(dt).double()

    va, vb = rnd((n, c, h, w)), rnd((n, c, h, w))
    W = rnd((c, c), c ** -0.5).float().double()
    gza, gzb = rnd((n, c, h, w)), rnd((n, c, h, w))
    refs = {}
    for emul in ((False, True) if dt == torch.bfloat16 else (False,)):
        var = va.to(cuda).requires_grad_(True)
        wr = W.to(cuda).requires_grad_(True)
        za, zb = _coatt_ref(var, vb.to(cuda), wr, emul)
        ((za * gza.to(cuda)).sum() + (zb * gzb.to(cuda)).sum()).backward()
        refs[emul] = {"Z_a": za.detach(), "Z_b": zb.detach(), "dV_a": var.grad, "dW": wr.grad}
    nhwc = lambda x: x.permute(0, 2, 3, 1).reshape(n * h * w, c)
    vag = nhwc(va).to(dt).to(cuda).contiguous().requires_grad_(True)
    vbg = nhwc(vb).to(dt).to(cuda).contiguous()
    Wg = W.float().to(cuda).requires_grad_(True)
    ga, gb = CoattFn.apply(vag, vbg, Wg, (n, h * w))
    torch.autograd.backward([ga, gb], [nhwc(gza).to(dt).to(cuda), nhwc(gzb).to(dt).to(cuda)])
    torch.cuda.synchronize()
    nchw = lambda t: t.reshape(n, h, w, c).permute(0, 3, 1, 2)
    got = {"Z_a": nchw(ga), "Z_b": nchw(gb), "dV_a": nchw(vag.grad), "dW": Wg.grad}
    rel = lambda a, b: ((a.double() - b.double()).abs().max() / b.double().abs().max()).item()
    for name in got:
        if dt == torch.float32:
            err = rel(got[name], refs[False][name])
            assert err <= 2e-4, (name, err)
        else:
            e_em, e_pure = rel(got[name], refs[True][name]), rel(got[name], refs[False][name])
            floor = rel(refs[True][name], refs[False][name])
            print("%s bf16: vs emul %.2e, vs pure %.2e, floor %.2e" % (name, e_em, e_pure, floor))
            assert e_em <= 3e-2 and e_pure <= 1.25 * floor + 2e-3, (name, e_em, e_pure, floor)


def test_configs1_473_b4_fp32_matches_reference(cuda):
    """configs[1] pinned to the REFERENCE itself: one fp32 train step (forward of both frames x
    both modalities, loss, backward) at 473 x 473 with 4 frame pairs, against the reference run
    in fp64 on the same inputs / weights (tests/golden/train_b4_473.npz, make_golden.py train473;
    rgbd_segmentation_RAA.py:139-268, train.py:595-599).  Floor rule of tests/test_gpu_model.py:
    outputs within 8x the reference's own fp32-vs-fp64 floor, masks identical outside the
    ambiguity band, gradient norms within max(8x own floor, p90 floor), gradient heads and BN
    buffers within 8x floor.  Outputs / features are compared on the fixture's subgrid."""
    from conftest import golden_meta
    z = golden("train_b4_473.npz")
    meta = golden_meta()["train_b4_473"]
    inp = synthetic_inputs(4, 473, 473, seed=1234)
    assert [zlib.crc32(t.numpy().tobytes()) for t in inp] == list(z["in_crc32"]), \
        "synthetic input generator drifted"
    inp = [t.to(cuda) for t in inp]
    m = make_model(cuda, torch.float32).train()
    stages = {}
    x1, x2, labels = m(*inp[:4], stages=stages)
    loss = L.bce_l1(x1, inp[4]) + L.bce_l1(x2, inp[5])
    loss.backward()
    torch.cuda.synchronize()
    n, h, w = stages["geo"]
    to_nchw = lambda t: t.float().view(n, h, w, -1).permute(0, 3, 1, 2)
    sub2 = (slice(None), slice(None), slice(None, None, 2), slice(None, None, 2))
    subf = (slice(None), slice(None, None, 8), slice(None, None, 3), slice(None, None, 3))
    for name, t, sub in (("x1", x1, sub2), ("x2", x2, sub2), ("labels", labels, sub2),
                         ("V_a", to_nchw(stages["V_a"]), subf), ("D_a", to_nchw(stages["D_a"]), subf)):
        ref = z["f64r/" + name].astype(np.float64)
        got = t.detach().double()[sub].cpu().numpy()
        floor = float(z["floor/" + name][0])
        tol = 8 * floor + 1e-5 * max(1.0, float(np.abs(ref).max()))
        err = float(np.abs(got - ref).max())
        assert err <= tol, "%s: max err %.3g > tol %.3g (floor %.3g)" % (name, err, tol, floor)
        if name in ("x1", "x2"):
            amb = np.abs(ref - 0.5) <= tol
            flips = ((got > 0.5) != (ref > 0.5)) & ~amb
            assert not flips.any(), (name, int(flips.sum()))
            full_mean = float(z["f64/mean/" + name][0])
            assert abs(t.double().mean().item() - full_mean) <= tol, name
    lref, lfloor = float(z["f64/loss"][0]), float(z["floor/loss"][0])
    assert abs(loss.item() - lref) <= 8 * lfloor + 1e-5 * abs(lref), (loss.item(), lref, lfloor)
    named = dict(m.named_parameters())
    norms = np.array([named[k].grad.double().norm().item() for k in meta["grad_norm_keys"]])
    ref = z["f64/grad_norm"]
    rel = np.abs(norms - ref) / np.maximum(ref, 1e-12)
    floor = np.abs(z["f32/grad_norm"] - ref) / np.maximum(ref, 1e-12)
    zero = ref < 1e-6 * np.median(ref)   # analytically zero (conv bias before a train-mode BN)
    # per tensor: 8x its own reference floor or the 99th percentile of the reference's floors
    # (a tensor whose reference fp32 error happens to be tiny is not held to that luck); and the
    # error DISTRIBUTION within 1.5x the reference's own fp32 one
    nz = ~zero
    tol = np.maximum(8 * floor, np.quantile(floor[nz], 0.99)) + 1e-3
    ok = (rel <= tol) | (zero & (norms < 1e-5 * np.median(ref)))
    for q in (0.5, 0.9):
        assert np.quantile(rel[nz], q) <= 1.5 * np.quantile(floor[nz], q) + 1e-4, q
    print("configs[1] fp32 grad-norm rel err vs fp64: median %.2e p90 %.2e max %.2e; reference's own "
          "fp32 floor: median %.2e p90 %.2e max %.2e" % (
              np.median(rel[nz]), np.quantile(rel[nz], 0.9), rel[nz].max(), np.median(floor[nz]),
              np.quantile(floor[nz], 0.9), floor[nz].max()))
    assert ok.all(), "grad norms off: %s" % [(meta["grad_norm_keys"][i], "%.2e" % rel[i], "%.2e" % tol[i])
                                              for i in np.nonzero(~ok)[0]][:8]
    for k in meta["select"]:
        g = named[k].grad.detach().double().flatten().cpu().numpy()
        r = z["f64/grad_head/" + k]
        fl = float(z["floor/grad_head/" + k][0])
        err = np.abs(g[:r.size] - r).max()
        assert err <= 8 * fl + 0.02 * np.abs(r).max(), (k, err, fl)
    sd = m.state_dict()
    for k in [f for f in z.files if f.startswith("f64/buf/")]:
        key = k[len("f64/buf/"):]
        got = sd[key].double().cpu().numpy()
        fl = float(z["floor/buf/" + key][0])
        assert np.abs(got - z[k]).max() <= 8 * fl + 1e-6 * max(1.0, np.abs(z[k]).max()), key


def _step_once(m, inp):
    x1, x2, _ = m(*inp[:4])
    loss = L.bce_l1(x1, inp[4]) + L.bce_l1(x2, inp[5])
    return x1, x2, loss


def _grad_norms(m):
    return np.array([p.grad.double().norm().item() for p in m.parameters() if p.grad is not None])


def test_configs1_473_b4_bf16_step_tracks_fp32(cuda):
    """configs[1]: 473 x 473, 4 frame pairs, bf16, fwd + loss + bwd on the HIP path, with the
    same inputs / weights through the fp32 HIP path as the yardstick (the fp32 path itself is
    pinned to the reference at this very configuration by the test above; bf16 blocks are pinned
    to fp64 in tests/test_gpu_blocks_bf16.py).
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


def test_configs1_473_b4_bf16_step_vs_reference(cuda):
    """configs[1] in bf16 against the REFERENCE's own run (tests/golden/train_b4_473.npz, the
    reference in fp64 at this very configuration), not against our fp32 path: the aggregates a
    training step consumes, with the bounds of test_configs1_473_b4_bf16_step_tracks_fp32 --
    |loss - loss_ref| <= 3 %, mean(x1), mean(x2) within 0.03, per-parameter gradient norms: median
    ratio within [0.8, 1.25] and >= 90 % of the parameters within [0.5, 2].  (Element parity is
    not the bar in bf16: the random-init 101-layer network is chaotic under bf16 rounding -- the
    reference itself run in bf16 agrees with its fp64 masks on ~80 % of pixels; bf16 blocks are
    pinned elementwise to fp64 in tests/test_gpu_blocks_bf16.py.)"""
    from conftest import golden_meta
    z = golden("train_b4_473.npz")
    meta = golden_meta()["train_b4_473"]
    inp = synthetic_inputs(4, 473, 473, seed=1234)
    assert [zlib.crc32(t.numpy().tobytes()) for t in inp] == list(z["in_crc32"])
    inp = [t.to(cuda) for t in inp]
    m = make_model(cuda, torch.bfloat16).train()
    x1, x2, loss = _step_once(m, inp)
    loss.backward()
    torch.cuda.synchronize()
    lref = float(z["f64/loss"][0])
    assert np.isfinite(loss.item()) and abs(loss.item() - lref) <= 0.03 * abs(lref), (loss.item(), lref)
    for name, t in (("x1", x1), ("x2", x2)):
        ref = float(z["f64/mean/" + name][0])
        assert abs(t.double().mean().item() - ref) <= 0.03, (name, t.double().mean().item(), ref)
    named = dict(m.named_parameters())
    norms = np.array([named[k].grad.double().norm().item() for k in meta["grad_norm_keys"]])
    ref = z["f64/grad_norm"]
    nz = ref >= 1e-6 * np.median(ref)          # analytically zero norms excluded
    ratio = norms[nz] / ref[nz]
    inside = ((ratio >= 0.5) & (ratio <= 2.0)).mean()
    print("bf16 vs reference fp64 at 473x473 B=4: loss %.5f / %.5f, grad-norm ratio median %.3f, "
          "%.1f %% within [0.5, 2]" % (loss.item(), lref, np.median(ratio), 100 * inside))
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
