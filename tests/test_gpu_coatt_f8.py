"""fp8 (MX e4m3) co-attention forward, BASELINE configs[4] (cn_coatt_f8_fwd): the affinity
S = Va_t Vb^T and the gathers P.V of both directions (rgbd_segmentation_RAA.py:160-170) on the
block-scaled MFMA.

Statistical parity with a stated tolerance, in two layers:
  * against fp64 on the kernel's OWN quantised operands (Va_t, Vb as rows with one E8M0
    exponent per 32 channels, V with one per channel and 32 consecutive keys, emulated here
    with torch's float8_e4m3fn): only the e4m3 rounding of P (<= 2^-4 relative per weight, rms
    2^-4/sqrt(3) = 3.6e-2) and fp32 accumulation remain -> relative L2 error <= 3e-2 (measured
    0.5-1.3e-2 at logit std 16, 2.1e-2 at std 4 where more weights matter), max error <= 8e-2
    of the output scale (a peaky row's output is one or two weights times V, so the max
    inherits the 2^-4);
  * against pure fp64 of the bf16 inputs (the reference's math) -- the fp8 floor of the block:
    this co-attention has no temperature, so the logits are S = Va_t . Vb over 256 channels (std
    ~16 for unit features) and 3 mantissa bits per operand move them by ~1, i.e. the softmax
    weights by ~e^(+-1): relative L2 error of Z measured 0.13-0.17 at logit std 16 (bound 0.25)
    and bound 0.12 at std 4.
The kernel serves the no-grad (inference) co-attention of the fp8 model; its training forward
is the bf16 flash kernel, whose backward recomputes P from that forward's own normalisers
(test_coattfn_fp8_flag_inference_only).
"""
import math

import pytest
import torch

from cosnet_amd import ops

pytestmark = pytest.mark.gpu


def make(n, hw, c, cuda, seed, scale=1.0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return [(torch.randn((n * hw, c), generator=g) * scale).to(torch.bfloat16).to(cuda) for _ in range(3)]


def _scale_of(amax):
    e = torch.ceil(torch.log2(amax / 448.0))
    e = torch.where(amax > 0, e, torch.zeros_like(e)).clamp(-126, 127)
    return torch.exp2(e)


def mx_rows(x):
    """[R, 256] -> dequantised MX rows (one E8M0 scale per 32 channels)."""
    r = x.shape[0]
    xb = x.double().reshape(r, 8, 32)
    sc = _scale_of(xb.abs().amax(-1))[..., None]
    return ((xb / sc).to(torch.float8_e4m3fn).double() * sc).reshape(r, 256)


def mx_vt(v, n, hw):
    """V [n*hw, 256] -> dequantised with one E8M0 scale per (channel, 32 consecutive keys of a
    64-key tile): the k-blocks of the scaled MFMA's PV product."""
    out = v.double().reshape(n, hw, 256).clone()
    for k0 in range(0, hw, 32):
        blk = out[:, k0:k0 + 32, :]
        sc = _scale_of(blk.abs().amax(1, keepdim=True))
        out[:, k0:k0 + 32, :] = (blk / sc).to(torch.float8_e4m3fn).double() * sc
    return out.reshape(n * hw, 256)


def ref(qa, a, b, n, hw):
    c = 256
    qa, a, b = qa.reshape(n, hw, c), a.reshape(n, hw, c), b.reshape(n, hw, c)
    S = qa @ b.transpose(1, 2)
    za = torch.softmax(S, dim=2) @ b
    zb = torch.softmax(S, dim=1).transpose(1, 2) @ a
    lse = torch.logsumexp(S, dim=2) / math.log(2)       # log2-sum-exp2 of S log2(e)
    return za.reshape(n * hw, c), zb.reshape(n * hw, c), lse


@pytest.mark.parametrize("n,hw,scale", [(2, 400, 1.0), (1, 97, 1.0), (1, 3600, 1.0), (2, 3600, 0.5)])
def test_coatt_f8_vs_fp64(cuda, n, hw, scale):
    c = 256
    vat, va, vb = make(n, hw, c, cuda, seed=hw, scale=scale)
    za = torch.empty((n * hw, c), dtype=torch.bfloat16, device=cuda)
    zb = torch.empty_like(za)
    lse_a = torch.empty((n, ops.hw_pad(hw)), dtype=torch.float32, device=cuda)
    lse_b = torch.empty_like(lse_a)
    ops.coatt_f8(vat, va, vb, n, hw, za, zb, lse_a, lse_b)
    torch.cuda.synchronize()
    assert torch.isfinite(za.float()).all() and torch.isfinite(zb.float()).all()
    # own-operand reference: rows of Va_t and Vb quantised, the gathered V's as V^T tiles
    qat, qb = mx_rows(vat), mx_rows(vb)
    qva, qvb = mx_vt(va, n, hw), mx_vt(vb, n, hw)
    S = qat.reshape(n, hw, c) @ qb.reshape(n, hw, c).transpose(1, 2)
    ra = (torch.softmax(S, dim=2) @ qvb.reshape(n, hw, c)).reshape(n * hw, c)
    rb = (torch.softmax(S, dim=1).transpose(1, 2) @ qva.reshape(n, hw, c)).reshape(n * hw, c)
    lse_ref = torch.logsumexp(S, dim=2) / math.log(2)
    rel = lambda g, r: ((g.double() - r).abs().max() / r.abs().max()).item()
    l2 = lambda g, r: ((g.double() - r).norm() / r.norm()).item()
    ea, eb = rel(za, ra), rel(zb, rb)
    la, lb = l2(za, ra), l2(zb, rb)
    assert la <= 3e-2 and lb <= 3e-2 and ea <= 8e-2 and eb <= 8e-2, (la, lb, ea, eb)
    el = (lse_a[:, :hw].double() - lse_ref).abs().max().item()
    assert el <= 2e-2 * max(1.0, lse_ref.abs().max().item() / 64), el
    assert torch.isinf(lse_a[:, hw:]).all()
    # pure fp64 of the bf16 inputs: the fp8 floor of the block
    pa, pb, _ = ref(vat.double(), va.double(), vb.double(), n, hw)
    fa, fb = l2(za, pa), l2(zb, pb)
    print("coatt fp8 n=%d hw=%d logit-std %.0f: vs own-operand fp64 L2 %.2e / %.2e max %.2e / %.2e,"
          " vs pure fp64 L2 %.2e / %.2e" % (n, hw, 16 * scale * scale, la, lb, ea, eb, fa, fb))
    bound = 0.25 if scale >= 1.0 else 0.12
    assert fa <= bound and fb <= bound, (fa, fb, bound)


def test_coattfn_fp8_flag_inference_only(cuda, monkeypatch):
    """CoattFn with fp8=True (the model's fp8 contexts) runs cn_coatt_f8_fwd for the no-grad
    forward only.  The training forward stays the bf16 flash kernel, so the backward's
    recomputed S and P (exp2(S log2e - lse)) are the ones the forward normalised: the fp8-mode
    gradient is bitwise the bf16-mode gradient (whose kernels are pinned against fp64 autograd
    in test_gpu_coatt_fused.py::test_flash_training_fwd_bwd_vs_fp64)."""
    from cosnet_amd.functions import CoattFn
    n, hw, c = 2, 200, 256
    va, vb, _ = make(n, hw, c, cuda, seed=3, scale=0.7)
    W0 = (torch.randn((c, c)) * c ** -0.5).to(cuda)
    calls = []
    real = ops.coatt_f8
    monkeypatch.setattr(ops, "coatt_f8", lambda *a, **k: calls.append(1) or real(*a, **k))
    with torch.no_grad():
        CoattFn.apply(va, vb, W0, (n, hw), None, True)
    assert calls == [1]
    grads = []
    for f8 in (True, False):
        W = torch.nn.Parameter(W0.clone())
        vg = va.clone().requires_grad_(True)
        za, zb = CoattFn.apply(vg, vb, W, (n, hw), None, f8)
        g = torch.Generator(device="cpu").manual_seed(11)
        dza = torch.randn(za.shape, generator=g).to(cuda, za.dtype)
        dzb = torch.randn(zb.shape, generator=g).to(cuda, zb.dtype)
        torch.autograd.backward([za, zb], [dza, dzb])
        torch.cuda.synchronize()
        grads.append((za.detach(), zb.detach(), vg.grad, W.grad))
    assert calls == [1]                       # the training forwards did not take the fp8 kernel
    for a, b in zip(*grads):
        assert torch.isfinite(a.float()).all() and torch.equal(a, b)
