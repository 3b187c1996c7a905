"""Fused co-attention forward (cn_coatt_fused_fwd, S never materialised) against

  * an fp64 restatement of rgbd_segmentation_RAA.py:160-170 on the same bf16-rounded inputs
    (S = Va_t Vb^T, S_column = softmax_j, S_row = softmax_i, Z_a = Vb . S_col, Z_b = Va . S_row),
  * the materialised-S HIP path (affinity GEMM + two-direction softmax + two gathers).

The fused kernel rounds the softmax weights to bf16 before the P.V product (as the
materialised bf16 path does), so the tolerance is 1.5e-2 of the output scale; the logits have
std ~16 (unscaled, realistic for trained features) so the softmax is peaky.
"""
import pytest
import torch

from cosnet_amd import _native as nv
from cosnet_amd import ops

pytestmark = pytest.mark.gpu

TOL = 1.5e-2


def ref64(vat, va, vb, n, hw):
    """fp64 on the device (test oracle arithmetic, not the product path)."""
    c = vat.shape[1]
    qa = vat[:, :c].double().reshape(n, hw, c)
    a = va[:, :c].double().reshape(n, hw, c)
    b = vb[:, :c].double().reshape(n, hw, c)
    S = qa @ b.transpose(1, 2)                    # [n, i, j]
    za = torch.softmax(S, dim=2) @ b              # rows i: softmax over j
    zb = torch.softmax(S, dim=1).transpose(1, 2) @ a
    return za.reshape(n * hw, c), zb.reshape(n * hw, c)


def make(n, hw, c, cuda, ld_extra=0, seed=0, scale=1.0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    def t(s):
        x = (torch.randn((n * hw, c + ld_extra), generator=g) * s).to(torch.bfloat16).to(cuda)
        return x[:, ld_extra:] if ld_extra else x
    # |S| std ~ scale^2 * sqrt(c): scale 0.5 -> ~4 ... 1.0 -> 16
    return t(scale), t(scale), t(scale)


def rel(got, ref):
    return ((got.double() - ref).abs().max() / ref.abs().max().clamp_min(1e-9)).item()


@pytest.mark.parametrize("n,hw", [(1, 1), (2, 63), (2, 64), (1, 65), (2, 127), (2, 128), (2, 169),
                                  (1, 300), (2, 1271), (1, 3600), (5, 3600)])
def test_fused_vs_fp64(cuda, n, hw):
    c = 256
    vat, va, vb = make(n, hw, c, cuda, seed=hw)
    za = torch.empty((n * hw, c), dtype=torch.bfloat16, device=cuda)
    zb = torch.empty_like(za)
    ops.coatt_fused(vat, va, vb, n, hw, za, zb)
    ra, rb = ref64(vat, va, vb, n, hw)
    torch.cuda.synchronize()
    assert torch.isfinite(za.float()).all() and torch.isfinite(zb.float()).all()
    ea, eb = rel(za, ra), rel(zb, rb)
    assert ea <= TOL and eb <= TOL, (ea, eb)


@pytest.mark.parametrize("scale", [0.25, 0.5, 1.0, 1.5])
def test_fused_logit_scales(cuda, scale):
    """From nearly uniform attention (S std ~1) to one-hot (std ~36): online rescale paths."""
    n, hw, c = 2, 700, 256
    vat, va, vb = make(n, hw, c, cuda, seed=7, scale=scale)
    za = torch.empty((n * hw, c), dtype=torch.bfloat16, device=cuda)
    zb = torch.empty_like(za)
    ops.coatt_fused(vat, va, vb, n, hw, za, zb)
    ra, rb = ref64(vat, va, vb, n, hw)
    torch.cuda.synchronize()
    assert rel(za, ra) <= TOL and rel(zb, rb) <= TOL, (rel(za, ra), rel(zb, rb))


def test_fused_strided_views_and_single_direction(cuda):
    """Channel-slice views (row stride 512, as concat buffers hand them over) and a NULL output."""
    n, hw, c = 2, 500, 256
    vat, va, vb = make(n, hw, c, cuda, ld_extra=256, seed=3)
    assert ops.ld(va) == 512 and va.data_ptr() % 16 == 0
    za = torch.empty((n * hw, c), dtype=torch.bfloat16, device=cuda)
    zb = torch.empty_like(za)
    ops.coatt_fused(vat, va, vb, n, hw, za, zb)
    ra, rb = ref64(vat, va, vb, n, hw)
    zb1 = torch.full_like(za, 7.0)
    ops.coatt_fused(vat, va, vb, n, hw, None, zb1)
    torch.cuda.synchronize()
    assert rel(za, ra) <= TOL and rel(zb, rb) <= TOL
    assert torch.equal(zb1, zb)


def test_fused_rejects_bad_shapes(cuda):
    n, hw = 1, 64
    vat, va, vb = make(n, hw, 128, cuda)
    za = torch.empty((n * hw, 128), dtype=torch.bfloat16, device=cuda)
    with pytest.raises(nv.NativeError):
        ops.coatt_fused(vat, va, vb, n, hw, za, za)   # C != 256


def test_coattfn_inference_uses_fused_and_matches_materialised(cuda, monkeypatch):
    """CoattFn under no_grad goes through the fused kernel; same result as the materialised
    HIP path (affinity GEMM + softmax kernels + gathers) within bf16 rounding of P."""
    from cosnet_amd.functions import CoattFn
    n, hw, c = 2, 3600, 256
    _, va, vb = make(n, hw, c, cuda, seed=11, scale=0.7)
    # an nn.Parameter like the model's similarity weight (requires_grad=True under no_grad)
    W = torch.nn.Parameter((torch.randn((c, c), generator=torch.Generator().manual_seed(5)) * c ** -0.5).to(cuda))
    calls = []
    real = ops.coatt_fused
    monkeypatch.setattr(ops, "coatt_fused", lambda *a, **k: calls.append(1) or real(*a, **k))
    with torch.no_grad():
        fa, fb = CoattFn.apply(va, vb, W, (n, hw))
        monkeypatch.setattr(ops, "COATT_FUSED", False)
        ma, mb = CoattFn.apply(va, vb, W, (n, hw))
    torch.cuda.synchronize()
    assert len(calls) == 1
    assert rel(fa, ma.double()) <= TOL and rel(fb, mb.double()) <= TOL, (rel(fa, ma.double()), rel(fb, mb.double()))


@pytest.mark.parametrize("n,hw", [(1, 97), (2, 169), (2, 1271), (4, 3600)])
@pytest.mark.parametrize("which", ["both", "a_only", "b_only"])
def test_flash_training_fwd_bwd_vs_fp64(cuda, n, hw, which):
    """CoattFn's training path in bf16 (flash forward with LSE + flash backward: S, P and dS never
    in HBM) against fp64 autograd of rgbd_segmentation_RAA.py:158-170 on the same bf16 inputs.
    which: gradient reaching Z_a only / Z_b only / both (the depth block's Z_b gets none).
    Tolerance 3e-2 of each output's scale (P, dS rounded to bf16 as the materialised path does)."""
    from cosnet_amd.functions import CoattFn
    c = 256
    g = torch.Generator().manual_seed(hw + n)
    va = (torch.randn((n * hw, c), generator=g) * 0.7).to(torch.bfloat16)
    vb = (torch.randn((n * hw, c), generator=g) * 0.7).to(torch.bfloat16)
    W = torch.randn((c, c), generator=g) * c ** -0.5
    ga = torch.randn((n * hw, c), generator=g).to(torch.bfloat16)
    gb = torch.randn((n * hw, c), generator=g).to(torch.bfloat16)
    # fp64 reference on the device (test arithmetic)
    var = va.double().to(cuda).requires_grad_(True)
    wr = W.double().to(cuda).requires_grad_(True)
    vat = (var @ wr.t()).reshape(n, hw, c)
    b3 = vb.double().to(cuda).reshape(n, hw, c)
    S = vat @ b3.transpose(1, 2)
    za_r = (torch.softmax(S, 2) @ b3).reshape(n * hw, c)
    zb_r = (torch.softmax(S, 1).transpose(1, 2) @ var.reshape(n, hw, c)).reshape(n * hw, c)
    outs, grads = [], []
    if which in ("both", "a_only"):
        outs.append(za_r); grads.append(ga.double().to(cuda))
    if which in ("both", "b_only"):
        outs.append(zb_r); grads.append(gb.double().to(cuda))
    torch.autograd.backward(outs, grads)
    # HIP flash path
    vag = va.to(cuda).requires_grad_(True)
    Wg = torch.nn.Parameter(W.to(cuda))
    za, zb = CoattFn.apply(vag, vb.to(cuda), Wg, (n, hw))
    outs, grads = [], []
    if which in ("both", "a_only"):
        outs.append(za); grads.append(ga.to(cuda))
    if which in ("both", "b_only"):
        outs.append(zb); grads.append(gb.to(cuda))
    torch.autograd.backward(outs, grads)
    torch.cuda.synchronize()
    for name, got, ref in (("Z_a", za, za_r), ("Z_b", zb, zb_r), ("dV_a", vag.grad, var.grad),
                           ("dW", Wg.grad, wr.grad)):
        e = rel(got, ref.detach())
        assert e <= 3e-2, (name, e)


def _need_variants(lib):
    """Variants 2-4 were measured slower and live only in the development library
    (make EXPERIMENTAL=1, loaded through COSNET_HIP_LIB); the product library refuses them."""
    if not lib.cn_build_experimental():
        assert lib.cn_coatt_force_variant(2) == -1
        pytest.skip("co-attention variants 2-4 are built only with EXPERIMENTAL=1")


@pytest.mark.parametrize("n,hw", [(1, 97), (2, 169), (1, 1271), (4, 3600), (5, 3600)])
def test_paired_wave_kernel_is_bitwise_the_four_wave_kernel(cuda, n, hw):
    """The 8-wave forward (coatt_fused2_k: wave pairs share 32 query rows and split the output
    channels, two waves per SIMD) runs each S element, softmax step and P.V sum with the same
    MFMA sequence as the 4-wave kernel: no-grad forward (incl. the key-split tail), training
    forward (LSE) and the PV backward kernel (per-key normaliser, accumulate) are bitwise equal."""
    lib = nv.load()
    _need_variants(lib)
    vat, va, vb = make(n, hw, 256, cuda, seed=hw + 7, scale=0.8)
    g = torch.Generator().manual_seed(n * hw)
    dzb = torch.randn((n * hw, 256), generator=g).to(torch.bfloat16).to(cuda)
    outs = []
    old = lib.cn_coatt_force_variant(1)
    try:
        for v in (1, 2):
            lib.cn_coatt_force_variant(v)
            za, zb = ops.coatt_fused(vat, va, vb, n, hw, torch.empty_like(va), torch.empty_like(va))
            la = torch.empty((n, ops.hw_pad(hw)), dtype=torch.float32, device=cuda)
            lb = torch.empty_like(la)
            ta, tb = torch.empty_like(va), torch.empty_like(va)
            ops.coatt_flash_fwd(vat, va, vb, n, hw, ta, tb, la, lb)
            pv = (torch.randn((n * hw, 256), generator=torch.Generator().manual_seed(3)) * 0.1) \
                .to(torch.bfloat16).to(cuda)
            nws = int(nv.query("cn_coatt_fused_workspace_bytes", n, hw, 1))
            ws = torch.empty((max(nws, 4) // 4,), dtype=torch.float32, device=cuda)
            nv.call("cn_coatt_flash_pv_ws", vat.data_ptr(), ops.ld(vat), vb.data_ptr(), ops.ld(vb),
                    dzb.data_ptr(), ops.ld(dzb), lb.data_ptr(), n, hw, 256, pv.data_ptr(), ops.ld(pv),
                    1, ws.data_ptr(), nws, nv.stream())
            torch.cuda.synchronize()
            outs.append([za, zb, ta, tb, la[:, :hw], lb[:, :hw], pv])
    finally:
        lib.cn_coatt_force_variant(old)
    for k, (x, y) in enumerate(zip(*outs)):
        assert torch.isfinite(x.float()).all(), k
        assert torch.equal(x, y), (k, (x.float() - y.float()).abs().max().item())


@pytest.mark.parametrize("var", [3, 4])
@pytest.mark.parametrize("n,hw", [(1, 1), (2, 63), (1, 97), (2, 169), (1, 1271), (4, 3600), (5, 3600)])
def test_split_pair_kernels(cuda, n, hw, var):
    """The wave-pair forward / PV kernels that split S between the two waves of a pair --
    variant 3 (coatt_fused3_k, 8 waves: the keys, 16x16x32 S products, pair-wise max / P
    exchange through LDS) and variant 4 (coatt_dsplit_k, 4 waves: the channels, 64 query rows
    per pair, partial S exchanged and added) -- against fp64 of rgbd_segmentation_RAA.py:
    160-170 (no-grad forward incl. the key-split tail), and against the 4-wave kernel: training
    forward's LSE to 1e-4 (only S's summation order differs) and the PV backward kernel within
    the bf16 output rounding."""
    lib = nv.load()
    _need_variants(lib)
    vat, va, vb = make(n, hw, 256, cuda, seed=hw + 11, scale=0.8)
    g = torch.Generator().manual_seed(n * hw + 1)
    dzb = torch.randn((n * hw, 256), generator=g).to(torch.bfloat16).to(cuda)
    outs = []
    old = lib.cn_coatt_force_variant(1)
    try:
        for v in (1, var):
            lib.cn_coatt_force_variant(v)
            za, zb = ops.coatt_fused(vat, va, vb, n, hw, torch.empty_like(va), torch.empty_like(va))
            la = torch.empty((n, ops.hw_pad(hw)), dtype=torch.float32, device=cuda)
            lb = torch.empty_like(la)
            ta, tb = torch.empty_like(va), torch.empty_like(va)
            ops.coatt_flash_fwd(vat, va, vb, n, hw, ta, tb, la, lb)
            pv = torch.zeros_like(va)
            nws = int(nv.query("cn_coatt_fused_workspace_bytes", n, hw, 1))
            ws = torch.empty((max(nws, 4) // 4,), dtype=torch.float32, device=cuda)
            nv.call("cn_coatt_flash_pv_ws", vat.data_ptr(), ops.ld(vat), vb.data_ptr(), ops.ld(vb),
                    dzb.data_ptr(), ops.ld(dzb), lb.data_ptr(), n, hw, 256, pv.data_ptr(), ops.ld(pv),
                    0, ws.data_ptr(), nws, nv.stream())
            torch.cuda.synchronize()
            outs.append([za, zb, ta, tb, la[:, :hw], lb[:, :hw], pv])
    finally:
        lib.cn_coatt_force_variant(old)
    ra, rb = ref64(vat, va, vb, n, hw)
    v3 = outs[1]
    for got, ref in ((v3[0], ra), (v3[1], rb), (v3[2], ra), (v3[3], rb)):
        assert torch.isfinite(got.float()).all()
        assert rel(got, ref) <= TOL, rel(got, ref)
    for k in (4, 5):
        assert (outs[0][k] - v3[k]).abs().max().item() <= 1e-4 * max(1.0, outs[0][k].abs().max().item())
    e = rel(v3[6], outs[0][6].double())
    assert torch.isfinite(v3[6].float()).all() and e <= 8e-3, e


def _run_variant(lib, v, vat, va, vb, dzb, n, hw, cuda, acc=0):
    """No-grad forward, training forward (LSE) and PV backward kernel under variant v."""
    old = lib.cn_coatt_force_variant(v)
    assert old != -1
    try:
        za, zb = ops.coatt_fused(vat, va, vb, n, hw, torch.empty_like(va), torch.empty_like(va))
        la = torch.empty((n, ops.hw_pad(hw)), dtype=torch.float32, device=cuda)
        lb = torch.empty_like(la)
        ta, tb = torch.empty_like(va), torch.empty_like(va)
        ops.coatt_flash_fwd(vat, va, vb, n, hw, ta, tb, la, lb)
        pv = (torch.randn((n * hw, 256), generator=torch.Generator().manual_seed(3)) * 0.1) \
            .to(torch.bfloat16).to(cuda) if acc else torch.zeros_like(va)
        nws = int(nv.query("cn_coatt_fused_workspace_bytes", n, hw, 1))
        ws = torch.empty((max(nws, 4) // 4,), dtype=torch.float32, device=cuda)
        nv.call("cn_coatt_flash_pv_ws", vat.data_ptr(), ops.ld(vat), vb.data_ptr(), ops.ld(vb),
                dzb.data_ptr(), ops.ld(dzb), lb.data_ptr(), n, hw, 256, pv.data_ptr(), ops.ld(pv),
                acc, ws.data_ptr(), nws, nv.stream())
        torch.cuda.synchronize()
    finally:
        lib.cn_coatt_force_variant(old)
    return [za, zb, ta, tb, la[:, :hw], lb[:, :hw], pv]


@pytest.mark.parametrize("acc", [0, 1])
@pytest.mark.parametrize("n,hw", [(1, 1), (2, 63), (1, 97), (2, 169), (1, 300), (1, 1271), (4, 3600),
                                  (5, 3600), (8, 3600)])
def test_q48_kernel(cuda, n, hw, acc):
    """Variant 5 (coatt_q48_k: 48 query rows per wave, Q in registers, 16x16x32 tiles, a fixed
    per-row reference maximum) against fp64 of rgbd_segmentation_RAA.py:160-170 (no-grad forward
    incl. its key-split plan, training forward) and against the 4-wave kernel (variant 1): LSE
    to 1e-4 (S's summation order differs), the PV backward kernel (plain and accumulating)
    within the bf16 output rounding.  8 pairs: more 192-row items (304) than CUs, each of the
    256 ranges then spans parts of two items."""
    lib = nv.load()
    vat, va, vb = make(n, hw, 256, cuda, seed=hw + 13, scale=0.8)
    g = torch.Generator().manual_seed(n * hw + 2)
    dzb = torch.randn((n * hw, 256), generator=g).to(torch.bfloat16).to(cuda)
    v1 = _run_variant(lib, 1, vat, va, vb, dzb, n, hw, cuda, acc)
    v5 = _run_variant(lib, 5, vat, va, vb, dzb, n, hw, cuda, acc)
    ra, rb = ref64(vat, va, vb, n, hw)
    for k, (got, ref) in enumerate(((v5[0], ra), (v5[1], rb), (v5[2], ra), (v5[3], rb))):
        assert torch.isfinite(got.float()).all(), k
        assert rel(got, ref) <= TOL, (k, rel(got, ref))
    for k in (4, 5):
        assert (v1[k] - v5[k]).abs().max().item() <= 1e-4 * max(1.0, v1[k].abs().max().item()), k
    e = rel(v5[6], v1[6].double())
    assert torch.isfinite(v5[6].float()).all() and e <= 8e-3, e


@pytest.mark.parametrize("n,hw", [(1, 300), (2, 1271), (4, 3600)])
def test_q48_row_maximum_growth(cuda, n, hw):
    """The q48 kernel fixes each row's softmax reference at its first key tile's maximum and
    redoes the workgroup (an S-only pass for the exact maxima, then again with them) when a lane's
    partial sum ends above 2^100, i.e. a later logit outgrew the reference by ~100 log2 units (~69
    in logits) or overflowed.  Keys 200-231 (a later tile) and, in the other direction, query
    features scaled x8 push the logits' growth far past that: the outputs still match fp64."""
    lib = nv.load()
    vat, va, vb = make(n, hw, 256, cuda, seed=hw + 17, scale=0.8)
    for t in (vb, vat, va):
        t.view(n, hw, 256)[:, 200:232] *= 8
    g = torch.Generator().manual_seed(n * hw + 4)
    dzb = torch.randn((n * hw, 256), generator=g).to(torch.bfloat16).to(cuda)
    v5 = _run_variant(lib, 5, vat, va, vb, dzb, n, hw, cuda)
    v1 = _run_variant(lib, 1, vat, va, vb, dzb, n, hw, cuda)
    ra, rb = ref64(vat, va, vb, n, hw)
    for k, (got, ref) in enumerate(((v5[0], ra), (v5[1], rb), (v5[2], ra), (v5[3], rb))):
        assert torch.isfinite(got.float()).all(), k
        assert rel(got, ref) <= TOL, (k, rel(got, ref))
    for k in (4, 5):
        assert (v1[k] - v5[k]).abs().max().item() <= 1e-4 * max(1.0, v1[k].abs().max().item()), k


@pytest.mark.parametrize("n,hw", [(4, 3600), (5, 3600)])
def test_q48_pv_split_partials_under_cancellation(cuda, n, hw):
    """The 48-row kernel's cut items store their un-normalised partial O rows in bf16 (round 5;
    the 4-wave kernel kept fp32).  In the PV backward kernel (dV_a += sum_j P1[i][j] dZb[j]) the
    gradient dZb has random signs, so segment partials can cancel and each partial's bf16 rounding
    is relative to the partial, not to the (smaller) result.  Worst case here: nearly flat
    softmaxes (features x 0.25: logit std ~1) and dZb = +-1 alternating over the keys, so each row
    sums ~3600 terms that cancel to ~1/60 of their magnitude.  Pinned against fp64 per row,
    relative to the row's magnitude scale sum_j P1[i][j] |dZb[j]| (the scale a partial's rounding
    is relative to): <= 2^-8 for the split plan; the 4-wave kernel (fp32 partials, only the final
    bf16 rounding) is measured beside it, and both errors relative to the row's own result are
    printed."""
    lib = nv.load()
    vat, va, vb = make(n, hw, 256, cuda, seed=hw + 29, scale=0.25)
    sgn = torch.where(torch.arange(n * hw) % 2 == 0, 1.0, -1.0)[:, None]
    g = torch.Generator().manual_seed(n * hw + 6)
    dzb = (sgn * (1.0 + 0.1 * torch.rand((n * hw, 256), generator=g))).to(torch.bfloat16).to(cuda)
    c = 256
    S = vat.double().reshape(n, hw, c) @ vb.double().reshape(n, hw, c).transpose(1, 2)
    P1 = torch.softmax(S, dim=1)                                   # over i for each key j
    d = dzb.double().reshape(n, hw, c)
    ref = (P1 @ d).reshape(n * hw, c)
    scale = (P1 @ d.abs()).reshape(n * hw, c)
    out = {}
    for v in (5, 1):
        pv = _run_variant(lib, v, vat, va, vb, dzb, n, hw, cuda)[6]
        err = (pv.double() - ref).abs()
        out[v] = ((err / scale).max().item(), (err.norm() / ref.norm()).item())
    print("PV under cancellation n=%d hw=%d: |ref|/scale %.3f; q48 (bf16 partials) max err/scale "
          "%.2e, rel L2 %.2e; 4-wave (fp32 partials) %.2e, %.2e" % (
              n, hw, (ref.abs() / scale).mean().item(), out[5][0], out[5][1], out[1][0], out[1][1]))
    assert out[5][0] <= 2 ** -8, out
