"""fp8 (OCP e4m3 / e5m2) path, BASELINE configs[4]: statistical parity with bf16.

The fp8 path changes the forward conv GEMM operands (e4m3), the dgrad operands of the
compute-heavy convs (e5m2 output gradients x e4m3 transposed weights) and -- for the no-grad
co-attention -- the affinity / gather operands (cosnet_amd/fp8.py); the training co-attention
stays the bf16 flash pair, so its gradient is the gradient of its forward.  Parity is
statistical, with the bounds DESIGN §3.5 states: over 4 seeded SGD steps
at 97x97 (B = 2 pairs), each on a different seeded batch, the mean fp8 loss within 5 % of the
mean bf16 loss, every step within 15 %, the step-0 gap (same weights: the forward's precision
alone) within 8 %, and the output maps' means within 0.03.  The distribution these bounds are
set against, 5 seeds x {fp32, bf16, fp8} (tools/fp8_curve_dist.py, profiles/r04_fp8_curve_dist.json):
mean gap 1.0-4.0 % (median 1.8 %), per-step gap median 4.1 %, p90 7.9 %, max 14.7 %, map-mean gap
<= 0.026 -- while bf16 itself is up to 18 % per step and 0.032 in map mean away from fp32 on the
same batches (this random-init 101-layer net is chaotic in low precision).  The kernels
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
    # this seed (100) in the committed distribution: step gaps 4.3 / 7.5 / 6.7 / 3.6 %, mean 1.3 %
    assert rel[0] <= 0.08, (l8, l16)     # same weights: the forward's precision alone
    assert abs(l8.mean() - l16.mean()) <= 0.05 * l16.mean() and (rel <= 0.15).all(), (l8, l16)
    assert abs(m8[0] - m16[0]) <= 0.03 and abs(m8[1] - m16[1]) <= 0.03, (m8, m16)
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
