"""fp8 (OCP e4m3 / e5m2) path, BASELINE configs[4]: statistical parity with bf16.

The fp8 path changes the forward conv GEMM operands (e4m3), the dgrad and 3x3 weight-gradient
operands of the compute-heavy convs (e5m2 output gradients x e4m3), and the co-attention's
affinity / gather operands (MX-fp8) in inference AND training -- the training backward
recomputes S and P from the fp8 forward's decoded operands and normalisers, so its gradient is
the gradient of its forward (tests/test_gpu_coatt_f8.py).  Parity is statistical (SURVEY.md §7
step 9), with the bounds DESIGN §3.5 states: over 4 seeded SGD steps at 97x97 (B = 2 pairs),
each on a different seeded batch, the mean fp8 loss within 5 % of the mean bf16 loss, every step
within 15 %, the step-0 gap (same weights: the forward's precision alone) within 8 %, and the
output maps' means within 0.045.  The distribution these bounds are set against, 8 seeds x
{fp32, bf16, fp8} of the round-6 path (tools/fp8_curve_dist.py, profiles/r06_fp8_curve_dist.json):
mean gap 0.4-3.7 % (median 1.0 %), per-step gap median 2.6 %, p90 6.0 %, max 7.7 % (round 4,
bf16 training co-attention: 4.1 / 7.9 / 14.7 %), map-mean gap <= 0.035 (round 4: 0.026) --
while bf16 itself is up to 7.9 % per step and 0.040 in map mean away from fp32 on the same
batches (this random-init 101-layer net is chaotic in low precision).  The map bound is the
bf16 path's own distance from fp32 on that distribution (0.040) plus 0.005: the fp8 affinity
moves the attention weights by ~e^(+-1) (logits of std ~16, 3 mantissa bits per operand), so
the trained maps sit further from bf16 than with the bf16 training co-attention of round 4.  The kernels
themselves are pinned exactly in test_gpu_kernels.py (test_fp8_quant_matches_torch_e4m3fn,
test_conv_fwd_fp8).
"""
import numpy as np
import pytest
import torch

import cosnet_amd as C
from cosnet_amd import ops
from cosnet_amd.init_recipe import recipe_state_dict, synthetic_inputs
from cosnet_amd.optim import SGD, reference_param_groups
from cosnet_amd.train_step import TrainStep

pytestmark = pytest.mark.gpu

STEPS = 4


def _run(cuda, fp8, graphed, size=97, batch=2):
    m = C.build_model(torch.bfloat16)
    m.load_state_dict(recipe_state_dict(m.state_dict()))
    m.encoder.main_classifier.requires_grad_(False)
    m = m.to(cuda).train()
    m.set_fp8(fp8)
    g0, g1 = reference_param_groups(m)
    opt = SGD([g0, g1], [2.5e-6, 2.5e-3], momentum=0.9, weight_decay=5e-4)
    step = TrainStep(m, opt, batch, size, graphed=graphed)
    losses, means = [], []
    for i in range(STEPS):
        ins = [t.to(cuda) for t in synthetic_inputs(batch, size, size, seed=100 + i)]
        step.load(*ins)
        if graphed and i == 1:
            step.capture(warmup=0)     # record after one eager step (states, tables exist)
        loss = step([2.5e-6, 2.5e-3]) if (graphed and i >= 1) else step.eager([2.5e-6, 2.5e-3])
        losses.append(loss.item())
    with torch.no_grad():
        x1, x2, _ = m(*[t.to(cuda) for t in synthetic_inputs(batch, size, size, seed=999)[:4]])
    torch.cuda.synchronize()
    return np.array(losses), (x1.mean().item(), x2.mean().item()), m


def test_fp8_training_loss_curve_tracks_bf16(cuda):
    l16, m16, _ = _run(cuda, False, False)
    l8, m8, model = _run(cuda, True, False)
    assert np.isfinite(l8).all()
    rel = np.abs(l8 - l16) / np.abs(l16)
    # this seed (100) in the committed distribution: step gaps 4.4 / 2.7 / 5.1 / 4.1 %, mean 1.0 %
    assert rel[0] <= 0.08, (l8, l16)     # same weights: the forward's precision alone
    assert abs(l8.mean() - l16.mean()) <= 0.05 * l16.mean() and (rel <= 0.15).all(), (l8, l16)
    # this seed in profiles/r06_fp8_curve_dist.json: 0.035 / 0.011
    assert abs(m8[0] - m16[0]) <= 0.045 and abs(m8[1] - m16[1]) <= 0.045, (m8, m16)
    ctx = model.fp8
    assert len(ctx.weights._c) > 100 and len(ctx.acts.slots) > 50   # the encoders ran fp8
    assert len(ctx.grads.slots) >= 20                                # and their dgrads (e5m2)


def test_fp8_graphed_step_matches_eager_fp8(cuda):
    """The recorded step (fp8 weight refresh + delayed activation scales inside the graph)
    reproduces the eager fp8 trajectory."""
    le, _, _ = _run(cuda, True, False)
    lg, _, _ = _run(cuda, True, True)
    assert np.allclose(le, lg, rtol=1e-3), (le, lg)


def test_configs4_fp8_b8_graphed_step(cuda):
    """BASELINE configs[4] per GPU: 8 frame pairs at 473 x 473 through the recorded fp8 step
    (e4m3 forward convs, e5m2 dgrads, bf16 weight gradients, fp32 masters): finite losses,
    parameters move, the fp8 states are live."""
    m = C.build_model(torch.bfloat16)
    m.load_state_dict(recipe_state_dict(m.state_dict()))
    m.encoder.main_classifier.requires_grad_(False)
    m = m.to(cuda).train()
    m.set_fp8(True)
    g0, g1 = reference_param_groups(m)
    opt = SGD([g0, g1], [2.5e-6, 2.5e-3], momentum=0.9, weight_decay=5e-4)
    step = TrainStep(m, opt, 8, 473)
    step.load(*[t.to(cuda) for t in synthetic_inputs(8, 473, 473, seed=1234)])
    step.capture(warmup=1)
    w0 = m.reduce_channels_A.weight.detach().clone()
    losses = [step([2.5e-6, 2.5e-3]).item() for _ in range(2)]
    torch.cuda.synchronize()
    assert all(np.isfinite(losses)), losses
    assert not torch.equal(w0, m.reduce_channels_A.weight.detach())
    for p in m.parameters():
        assert torch.isfinite(p).all()
    assert len(m.fp8.grads.slots) >= 20 and len(m.fp8.acts.slots) > 50
    st = m.fp8.grads.states[:len(m.fp8.grads.slots)]
    assert torch.isfinite(st).all() and (st[:, 0] > 0).all() and (st[:, 3] == 57344).all()


def test_fp8_weight_gradient_of_bottleneck_matches_its_operands(cuda, monkeypatch):
    """configs[4] fp8 weight gradient inside the bottleneck backward (a layer-3 block at the
    configs[1] training shape, encoder_fn.bottleneck_fwd / bottleneck_bwd with the grouped
    WgradQueue): conv2's dW = e5m2 dc2 (the copy its fp8 dgrad quantises) x the e4m3 y1 copy the
    fp8 forward conv read, dequantised with the scale y1 was quantised with -- the forward pass's
    snapshot, although end() has advanced the live scale since.  Equal to fp64 of the decoded
    operands (2e-3 of the max: fp32 accumulation only).  Against fp64 of the SAME backward's bf16
    operands (what the bf16 weight gradient computes) it may differ only by the operand
    quantisation itself -- the distance between the two fp64 references, measured in the test
    (e5m2 keeps 2 mantissa bits: 0.073 relative L2 on this block), plus the kernel's 2e-3."""
    from cosnet_amd import encoder_fn as E
    n1, h, w = 4, 60, 60
    m = C.build_model(torch.bfloat16)
    m.load_state_dict(recipe_state_dict(m.state_dict()))
    m = m.to(cuda).train()
    m.set_fp8(True)
    m._set_dtype()
    ctx = m.fp8
    blk = m.encoder.backbone.layer3[5]
    g = torch.Generator().manual_seed(21)
    x = torch.relu(torch.randn((2 * n1 * h * w, 1024), generator=g)).to(torch.bfloat16).to(cuda)
    dy = (torch.randn((n1 * h * w, 1024), generator=g) * 0.1).to(torch.bfloat16).to(cuda)
    monkeypatch.setattr(E, "WGRAD_FP8", True)
    ctx.acts.begin()
    rec = []
    E.bottleneck_fwd(blk, x, (2 * n1, h, w), 2, rec)
    ctx.acts.end()
    ctx.grads.begin()
    grads, wq = E.GradSink(), E.WgradQueue()
    E.bottleneck_bwd(rec[0], dy, grads, wq=wq)
    wq.flush()
    torch.cuda.synchronize()
    dw2 = grads[blk.conv2.weight].detach().double().cpu()
    x8, handle, slot = rec[0][2][16][0]          # conv2's saved e4m3 input (Fp8Acts.saved)
    sx = handle.state(slot)[0].item()
    dys = [v for v in ctx.grads.pass_cache.values() if tuple(v[0].shape) == (n1 * h * w, 256)]
    assert len(dys) == 1, [tuple(v[0].shape) for v in ctx.grads.pass_cache.values()]
    dy8, ds = dys[0][0], dys[0][1][0].item()

    def wgrad64(xa, da):
        xp = torch.nn.functional.pad(xa, (0, 0, 2, 2, 2, 2))
        ref = torch.empty((256, 256, 3, 3), dtype=torch.float64)
        for r in range(3):
            for s in range(3):
                ref[:, :, r, s] = da.t() @ xp[:, 2 * r:2 * r + h, 2 * s:2 * s + w, :].reshape(-1, 256)
        return ref
    ref = wgrad64(x8[:n1 * h * w].cpu().view(torch.float8_e4m3fn).double().view(n1, h, w, 256) * sx,
                  dy8.cpu().view(torch.float8_e5m2).double().view(n1 * h * w, 256) * ds)
    err = ((dw2 - ref).abs().max() / ref.abs().max()).item()
    assert err <= 2e-3, err
    # the same backward's bf16 operands: y1 (frame a) and dc2 (the tensor dy8 quantises)
    y1 = rec[0][2][2][:n1 * h * w]
    ref16 = wgrad64(y1.double().cpu().view(n1, h, w, 256), dys[0][2].double().cpu())
    qerr = ((ref - ref16).norm() / ref16.norm()).item()
    assert 0 < qerr <= 0.15, qerr
    e16 = ((dw2 - ref16).norm() / ref16.norm()).item()
    assert e16 <= qerr + 2e-3, (e16, qerr)
    ctx.grads.end()


def test_fp8_vs_bf16_weight_gradient_with_pinned_scales(cuda, monkeypatch):
    """The bf16-vs-fp8 weight-gradient comparison of round 5's two-pass test, restored with the
    scale states pinned.  That test ran the block twice on one fp8 context (conv2's weight
    gradient fp8, then bf16) and failed at 0.166 against its bound 1.25 x 0.073 + 0.02
    (gpurun_out/r5d/01_tests.log:398): between the passes the context's delayed scales had
    moved -- Fp8Acts.end() / grads.end() of pass 1 advanced every activation and gradient scale,
    and pass 1 had CALIBRATED them (a first use quantises with the tensor's own amax) while pass
    2 quantised with the advanced delayed scales -- so pass 2's forward fp8 convs, its fp8
    dgrads and hence its y1 and dc2 were different operands, and the comparison measured two
    independent fp8 quantisations of the whole block, not the weight gradient's precision.  Here
    both passes start from the same fresh scale state (as pass 1 did), so y1 and dc2 are bitwise
    equal across them and the two weight gradients differ only by conv2's operand format:
    |fp8 - bf16| <= the operand quantisation distance measured on these operands + 2e-3."""
    from cosnet_amd import encoder_fn as E
    n1, h, w = 4, 60, 60
    m = C.build_model(torch.bfloat16)
    m.load_state_dict(recipe_state_dict(m.state_dict()))
    m = m.to(cuda).train()
    m.set_fp8(True)
    m._set_dtype()
    ctx = m.fp8
    blk = m.encoder.backbone.layer3[5]
    g = torch.Generator().manual_seed(21)
    x = torch.relu(torch.randn((2 * n1 * h * w, 1024), generator=g)).to(torch.bfloat16).to(cuda)
    dy = (torch.randn((n1 * h * w, 1024), generator=g) * 0.1).to(torch.bfloat16).to(cuda)
    out = {}
    for on in (True, False):
        for a in (ctx.acts, ctx.grads):   # pin: every pass starts from the same (fresh) scales
            a.states, a.slots, a.calibrated, a.pass_cache = None, {}, set(), {}
        monkeypatch.setattr(E, "WGRAD_FP8", on)
        ctx.acts.begin()
        rec = []
        E.bottleneck_fwd(blk, x, (2 * n1, h, w), 2, rec)
        ctx.acts.end()
        ctx.grads.begin()
        grads, wq = E.GradSink(), E.WgradQueue()
        E.bottleneck_bwd(rec[0], dy, grads, wq=wq)
        wq.flush()
        torch.cuda.synchronize()
        dys = [v for v in ctx.grads.pass_cache.values() if tuple(v[0].shape) == (n1 * h * w, 256)]
        assert len(dys) == 1
        out[on] = (grads[blk.conv2.weight].detach().double().cpu(), rec[0][2][2][:n1 * h * w].clone(),
                   dys[0][2].clone(), rec[0][2][16][0] if on else None, dys[0][0].clone(),
                   dys[0][1][0].item())
        ctx.grads.end()
    (dw8, y1a, dca, q2, dy8, ds), (dw16, y1b, dcb, _, _, _) = out[True], out[False]
    # the pinned scales reproduce the forward and the dgrad chain bit for bit
    assert torch.equal(y1a, y1b) and torch.equal(dca, dcb)
    x8, handle, slot = q2
    sx = handle.state(slot)[0].item()

    def wgrad64(xa, da):
        xp = torch.nn.functional.pad(xa, (0, 0, 2, 2, 2, 2))
        ref = torch.empty((256, 256, 3, 3), dtype=torch.float64)
        for r in range(3):
            for s in range(3):
                ref[:, :, r, s] = da.t() @ xp[:, 2 * r:2 * r + h, 2 * s:2 * s + w, :].reshape(-1, 256)
        return ref
    ref8 = wgrad64(x8[:n1 * h * w].cpu().view(torch.float8_e4m3fn).double().view(n1, h, w, 256) * sx,
                   dy8.cpu().view(torch.float8_e5m2).double().view(n1 * h * w, 256) * ds)
    ref16 = wgrad64(y1a.double().cpu().view(n1, h, w, 256), dca.double().cpu())
    qerr = ((ref8 - ref16).norm() / ref16.norm()).item()
    e = ((dw8 - dw16).norm() / dw16.norm()).item()
    e16 = ((dw16 - ref16).norm() / ref16.norm()).item()
    print("fp8 vs bf16 weight gradient: %.4f, operand quantisation %.4f, bf16 vs fp64 %.2e" % (e, qerr, e16))
    assert e16 <= 1e-2, e16                  # the bf16 weight gradient of these operands
    assert 0 < e <= qerr + 2e-3 + e16, (e, qerr, e16)
