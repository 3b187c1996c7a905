"""Per-kernel parity on the GPU: every libcosnet_hip kernel against a plain PyTorch fp64 CPU
restatement of the same aten op (the reference's own arithmetic), in both compute dtypes.

bf16 cases round the inputs to bf16 first, so the remaining error is fp32 accumulation plus
one bf16 output rounding: tolerance 1.2e-2 relative to the output scale; fp32 cases use the
exact f32-input MFMA: 2e-5 relative.
"""
import pytest
import torch
import torch.nn.functional as F

from cosnet_amd import _native as nv
from cosnet_amd import ops

pytestmark = pytest.mark.gpu

TOL = {torch.float32: 2e-5, torch.bfloat16: 1.2e-2}


def nhwc(x):  # NCHW -> [P, C]
    n, c, h, w = x.shape
    return x.permute(0, 2, 3, 1).reshape(n * h * w, c)


def nchw(x2d, n, h, w):
    return x2d.reshape(n, h, w, -1).permute(0, 3, 1, 2)


def close(got, ref, dt, scale=None):
    got = got.double().cpu()
    ref = ref.double().cpu()
    s = scale if scale is not None else max(ref.abs().max().item(), 1e-6)
    err = (got - ref).abs().max().item() / s
    assert err <= TOL[dt], "rel err %.3g > %.3g" % (err, TOL[dt])
    return err


def rnd(shape, dt, seed, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(shape, generator=g, dtype=torch.float64) * scale).to(dt).double()


CONV_CASES = [
    # n, cin, h, w, cout, k, stride, pad, dil
    (2, 64, 13, 11, 128, 1, 1, 0, 1),
    (2, 64, 13, 11, 64, 3, 1, 1, 1),
    (2, 32, 15, 9, 64, 3, 1, 2, 2),
    (2, 256, 7, 9, 128, 1, 2, 0, 1),
    (2, 8, 29, 31, 64, 7, 2, 3, 1),
    (1, 64, 9, 9, 512, 3, 1, 6, 6),
    (1, 320, 5, 6, 256, 3, 1, 1, 1),
    (3, 16, 4, 4, 8, 3, 1, 1, 1),
    # output rows longer than one K tile: the weight gradient's row-aligned K (gemm.h ConvGeom::kt)
    # walks several tiles per row, the later ones starting mid-row
    (2, 16, 6, 150, 32, 3, 1, 1, 1),
    (1, 8, 5, 141, 16, 3, 2, 1, 1),
]


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd_dgrad_wgrad(cuda, dt, case):
    n, cin, h, w, cout, k, s, p, d = case
    x = rnd((n, cin, h, w), dt, 1)
    wt = rnd((cout, cin, k, k), dt, 2, scale=(2.0 / (cin * k * k)) ** 0.5)
    b = rnd((cout,), torch.float32, 3)
    y_ref = F.conv2d(x, wt, b, s, p, d)
    oh, ow = y_ref.shape[2:]
    xg = nhwc(x).to(dt).to(cuda).contiguous()
    wp = wt.float().to(cuda).contiguous(memory_format=torch.channels_last)
    wf, wtt = ops.WCACHE.get(wp, dt)
    y, oh2, ow2 = ops.conv_fwd(xg, n, h, w, wf, cout, k, s, p, d, bias=b.float().to(cuda))
    assert (oh2, ow2) == (oh, ow)
    torch.cuda.synchronize()
    close(nchw(y, n, oh, ow), y_ref, dt)
    # backward
    gy = rnd(y_ref.shape, dt, 4)
    xr = x.clone().requires_grad_(True)
    wr = wt.clone().requires_grad_(True)
    F.conv2d(xr, wr, None, s, p, d).backward(gy)
    gyg = nhwc(gy).to(dt).to(cuda).contiguous()
    dw = ops.conv_wgrad(xg, n, h, w, cin, gyg, oh, ow, cout, k, s, p, d)
    torch.cuda.synchronize()
    close(ops.as_param_grad(dw, wp), wr.grad, dt)
    if s == 1 or k == 1:
        dx = ops.conv_dgrad(gyg, n, oh, ow, wtt, cin, k, s, p, d, h, w)
        torch.cuda.synchronize()
        close(nchw(dx, n, h, w), xr.grad, dt)
        # accumulate mode adds onto an existing gradient
        dx2 = ops.conv_dgrad(gyg, n, oh, ow, wtt, cin, k, s, p, d, h, w, out=dx.clone(), accumulate=True)
        torch.cuda.synchronize()
        close(nchw(dx2, n, h, w), 2 * xr.grad, dt)


@pytest.mark.parametrize("case", [(2, 2048, 9, 9, 256, 3, 1, 1, 1), (2, 2560, 7, 8, 64, 3, 1, 1, 1)])
def test_conv_fwd_split_k(cuda, case):
    """Deep one-round forward convs (the ASPP bottleneck shape class, K >= 16384, Cout <= 256) run
    on 256x256 tiles split over K + a fixed-order bf16 reduce with the bias; conv_fwd_bn's
    statistics then come from a pass over the reduced output.  Against torch fp64."""
    n, cin, h, w, cout, k, s, p, d = case
    dt = torch.bfloat16
    x = rnd((n, cin, h, w), dt, 61)
    wt = rnd((cout, cin, k, k), dt, 62, scale=(2.0 / (cin * k * k)) ** 0.5)
    b = rnd((cout,), torch.float32, 63)
    y_ref = F.conv2d(x, wt, b, s, p, d)
    oh, ow = y_ref.shape[2:]
    xg = nhwc(x).to(dt).to(cuda).contiguous()
    assert ops.fwd_split_floats(xg, n * oh * ow, cout, k * k * cin) > 0
    wp = wt.float().to(cuda).contiguous(memory_format=torch.channels_last)
    wf, _ = ops.WCACHE.get(wp, dt)
    y, _, _ = ops.conv_fwd(xg, n, h, w, wf, cout, k, s, p, d, bias=b.float().to(cuda))
    y2, _, _ = ops.conv_fwd(xg, n, h, w, wf, cout, k, s, p, d, bias=b.float().to(cuda))
    torch.cuda.synchronize()
    close(nchw(y, n, oh, ow), y_ref, dt)
    assert torch.equal(y, y2)
    bn = _bn_mod(cout, cuda, 64)
    yb, _, _, (mean, invstd) = ops.conv_fwd_bn(xg, n, h, w, wf, cout, k, s, p, d, bn, nseg=1,
                                               bias=b.float().to(cuda))
    torch.cuda.synchronize()
    assert torch.equal(yb, y)
    yd = nchw(y, n, oh, ow).double().cpu()
    m_ref = yd.mean(dim=(0, 2, 3))
    v_ref = yd.var(dim=(0, 2, 3), unbiased=False)
    assert torch.allclose(mean.double().cpu(), m_ref, rtol=1e-4, atol=1e-4 * m_ref.abs().max().item())
    assert torch.allclose(invstd.double().cpu(), 1 / torch.sqrt(v_ref + bn.eps), rtol=1e-3)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", [(2, 64, 13, 11, 128, 1, 1, 0, 1), (2, 32, 15, 9, 64, 3, 1, 2, 2),
                                  (2, 256, 7, 9, 128, 1, 2, 0, 1), (1, 64, 9, 9, 512, 3, 1, 6, 6),
                                  (1, 512, 12, 12, 512, 3, 1, 1, 1)])   # 256x128 tiles (>= 160 blocks)
def test_conv_wgrad_grouped(cuda, dt, case):
    """G weight gradients of one conv shape in one launch (the bottlenecks' grouped wgrads, no
    split-K): each problem against torch fp64; the launch is deterministic."""
    n, cin, h, w, cout, k, s, p, d = case
    G = 3
    oh, ow = ops.out_hw(h, w, k, s, p, d)
    jobs, refs = [], []
    for g in range(G):
        x = rnd((n, cin, h, w), dt, 40 + g)
        gy = rnd((n, cout, oh, ow), dt, 50 + g)
        wr = torch.zeros((cout, cin, k, k), dtype=torch.float64, requires_grad=True)
        F.conv2d(x, wr, None, s, p, d).backward(gy)
        refs.append(wr.grad)
        dw = torch.empty((cout, k * k * cin), dtype=torch.float32, device=cuda)
        jobs.append((nhwc(x).to(dt).to(cuda).contiguous(), nhwc(gy).to(dt).to(cuda).contiguous(), dw))
    ops.conv_wgrad_grouped(jobs, n, h, w, cin, oh, ow, cout, k, s, p, d)
    first = [dw.clone() for _, _, dw in jobs]
    ops.conv_wgrad_grouped(jobs, n, h, w, cin, oh, ow, cout, k, s, p, d)
    torch.cuda.synchronize()
    wp = torch.empty((cout, cin, k, k), device=cuda).contiguous(memory_format=torch.channels_last)
    for (_, _, dw), f, ref in zip(jobs, first, refs):
        close(ops.as_param_grad(dw, wp), ref, dt)
        assert torch.equal(dw, f)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", [(4, 64, 30, 30, 128, 1, 1, 0, 1), (2, 32, 40, 40, 64, 3, 1, 1, 1),
                                  (4, 128, 30, 30, 512, 1, 1, 0, 1), (2, 64, 36, 36, 64, 3, 1, 2, 2)])
@pytest.mark.parametrize("G", [2, 4])
def test_conv_wgrad_grouped_split(cuda, dt, case, G):
    """The small-shape groups split over K as well (cn_conv_wgrad_grouped_ws: G x nsplit blocks
    into per-problem slabs, one reduce launch): each problem against torch fp64; deterministic;
    the shapes are chosen so the split path runs (workspace > 0)."""
    n, cin, h, w, cout, k, s, p, d = case
    oh, ow = ops.out_hw(h, w, k, s, p, d)
    assert nv.query("cn_conv_wgrad_grouped_workspace_floats", ops.dtc(torch.empty(0, dtype=dt)), G, n,
                    oh, ow, cout, k, k, cin) > 0
    jobs, refs = [], []
    for g in range(G):
        x = rnd((n, cin, h, w), dt, 60 + g)
        gy = rnd((n, cout, oh, ow), dt, 70 + g)
        wr = torch.zeros((cout, cin, k, k), dtype=torch.float64, requires_grad=True)
        F.conv2d(x, wr, None, s, p, d).backward(gy)
        refs.append(wr.grad)
        dw = torch.full((cout, k * k * cin), float("nan"), dtype=torch.float32, device=cuda)
        jobs.append((nhwc(x).to(dt).to(cuda).contiguous(), nhwc(gy).to(dt).to(cuda).contiguous(), dw))
    ops.conv_wgrad_grouped(jobs, n, h, w, cin, oh, ow, cout, k, s, p, d, split=True)
    first = [dw.clone() for _, _, dw in jobs]
    ops.conv_wgrad_grouped(jobs, n, h, w, cin, oh, ow, cout, k, s, p, d, split=True)
    torch.cuda.synchronize()
    wp = torch.empty((cout, cin, k, k), device=cuda).contiguous(memory_format=torch.channels_last)
    for (_, _, dw), f, ref in zip(jobs, first, refs):
        close(ops.as_param_grad(dw, wp), ref, dt)
        assert torch.equal(dw, f)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("la,lb", [(0, 0), (0, 2), (2, 2)])
def test_gemm_layouts_batched(cuda, dt, la, lb):
    B, M, N, K = 3, 77, 136, 200
    a = rnd((B, M, K), dt, 5)
    bm = rnd((B, N, K), dt, 6)
    ref = torch.einsum("bmk,bnk->bmn", a, bm)
    # stored layouts: KC -> [M][K] rows; MC -> [K][M] rows (pad leading dims to multiples of 8)
    def store(t, lay, rows):
        if lay == 0:
            ldv = (t.shape[2] + 7) // 8 * 8
            buf = torch.zeros((B, t.shape[1], ldv), dtype=dt)
            buf[:, :, :t.shape[2]] = t.to(dt)
            return buf.to(cuda), ldv, t.shape[1] * ldv
        ldv = (rows + 7) // 8 * 8
        buf = torch.zeros((B, t.shape[2], ldv), dtype=dt)
        buf[:, :, :rows] = t.transpose(1, 2).to(dt)
        return buf.to(cuda), ldv, t.shape[2] * ldv
    A, lda, abs_ = store(a, la, M)
    Bt, ldb, bbs = store(bm, lb, N)
    out = torch.empty((B * M, N), dtype=torch.float32, device=cuda)
    ops.gemm(A, Bt, M, N, K, layout_a=la, layout_b=lb, lda=lda, ldb=ldb, a_bs=abs_, b_bs=bbs,
             out=out, ldc=N, c_bs=M * N, batch=B)
    torch.cuda.synchronize()
    close(out.view(B, M, N), ref, dt)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_gemm_splitk_atomic(cuda, dt):
    M, N, K = 256, 192, 4000
    a = rnd((K, M), dt, 7)
    b = rnd((K, N), dt, 8)
    ref = a.t() @ b
    out = torch.zeros((M, N), dtype=torch.float32, device=cuda)
    ops.gemm(a.to(dt).to(cuda), b.to(dt).to(cuda), M, N, K, layout_a=2, layout_b=2, lda=M, ldb=N,
             out=out, ldc=N, c_mode=1, nsplit=7)
    torch.cuda.synchronize()
    close(out, ref, dt)


def _bn_mod(c, cuda, seed):
    bn = torch.nn.BatchNorm2d(c).to(cuda)
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        bn.weight.copy_(1 + 0.1 * torch.randn(c, generator=g))
        bn.bias.copy_(0.1 * torch.randn(c, generator=g))
        bn.running_mean.copy_(0.2 * torch.randn(c, generator=g))
        bn.running_var.copy_(1 + 0.3 * torch.rand(c, generator=g))
    return bn


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("act", [0, 1, 2])
@pytest.mark.parametrize("c", [64, 320, 2560])
def test_batchnorm_train(cuda, dt, act, c):
    n, h, w = 2, 5, 7
    x = (rnd((n, c, h, w), dt, 9, scale=2.0) + 0.5).to(dt).double()
    bn = _bn_mod(c, cuda, 10)
    rm0, rv0 = bn.running_mean.double().cpu().clone(), bn.running_var.double().cpu().clone()
    xr = x.clone().requires_grad_(True)
    gw = bn.weight.detach().double().cpu().requires_grad_(True)
    gb = bn.bias.detach().double().cpu().requires_grad_(True)
    pw = torch.tensor([0.25], dtype=torch.float64, requires_grad=True)
    rm, rv = rm0.clone(), rv0.clone()
    y = F.batch_norm(xr, rm, rv, gw, gb, True, 0.1, 1e-5)
    y = F.relu(y) if act == 1 else (F.prelu(y, pw) if act == 2 else y)
    gy = rnd(y.shape, dt, 11)
    y.backward(gy)
    xg = nhwc(x).to(dt).to(cuda).contiguous()
    st = ops.bn_stats(xg, bn, True)
    prelu = torch.tensor([0.25], dtype=torch.float32, device=cuda)
    yg = ops.bn_apply(xg, st, bn, act=act, prelu=prelu)
    torch.cuda.synchronize()
    close(nchw(yg, n, h, w), y.detach(), dt)
    close(bn.running_mean, rm, torch.float32, scale=1.0)
    close(bn.running_var, rv, torch.float32, scale=1.0)
    gyg = nhwc(gy).to(dt).to(cuda).contiguous()
    dx, dgam, dbet, dpr = ops.bn_bwd(xg, gyg, yg, st, bn, act=act, prelu=prelu)
    torch.cuda.synchronize()
    close(nchw(dx, n, h, w), xr.grad, dt)
    close(dgam, gw.grad, dt)
    close(dbet, gb.grad, dt)
    if act == 2:
        close(dpr, pw.grad, dt)
    if act == 1:
        # the ReLU mask recomputed from x (no read of the activation) is bit-identical
        dx3, dgam3, dbet3, _ = ops.bn_bwd(xg, gyg, None, st, bn, act=1)
        torch.cuda.synchronize()
        assert torch.equal(dx3, dx) and torch.equal(dgam3, dgam) and torch.equal(dbet3, dbet)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_batchnorm_residual_forms(cuda, dt):
    n, c, h, w = 2, 64, 6, 5
    x = rnd((n, c, h, w), dt, 12)
    xd = rnd((n, c, h, w), dt, 13)
    res = rnd((n, c, h, w), dt, 14)
    bn, bnd = _bn_mod(c, cuda, 15), _bn_mod(c, cuda, 16)
    xg, xdg, rg = (nhwc(t).to(dt).to(cuda).contiguous() for t in (x, xd, res))
    st = ops.bn_stats(xg, bn, True)
    std = ops.bn_stats(xdg, bnd, True)
    y1 = ops.bn_apply(xg, st, bn, act=1, res=rg)
    y2 = ops.bn_apply(xg, st, bn, act=1, xr=xdg, rstats=std, rbn=bnd)
    ref_bn = lambda t, m: F.batch_norm(t, None, None, m.weight.detach().double().cpu(),
                                       m.bias.detach().double().cpu(), True, 0.1, 1e-5)
    torch.cuda.synchronize()
    close(nchw(y1, n, h, w), F.relu(ref_bn(x, bn) + res), dt)
    close(nchw(y2, n, h, w), F.relu(ref_bn(x, bn) + ref_bn(xd, bnd)), dt)
    # ReLU mask bits written by the apply (the bottleneck's residual BN): exactly y > 0 of the
    # stored values, and the backward from the bits (act 4) bitwise equal to the one re-reading y
    mk = ops.relu_mask(xg.shape[0], c, xg)
    y3 = ops.bn_apply(xg, st, bn, act=1, res=rg, mask=mk)
    vec = 8 if dt == torch.bfloat16 else 4
    bits = torch.stack([(mk.long() >> v) & 1 for v in range(vec)], dim=2).reshape(xg.shape[0], c)
    torch.cuda.synchronize()
    assert torch.equal(y3, y1) and torch.equal(bits.bool(), y1 > 0)
    gy = rnd((n, c, h, w), dt, 19)
    gyg = nhwc(gy).to(dt).to(cuda).contiguous()
    dres1, dres4 = torch.empty_like(xg), torch.empty_like(xg)
    d1 = ops.bn_bwd(xg, gyg, y1, st, bn, act=1, dres=dres1)
    d4 = ops.bn_bwd(xg, gyg, mk, st, bn, act=4, dres=dres4)
    torch.cuda.synchronize()
    assert all(torch.equal(a, b) for a, b in zip(d1[:3], d4[:3])) and torch.equal(dres1, dres4)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("c", [8, 256, 384])
def test_batchnorm_segments(cuda, dt, c):
    """Two frames stacked in one [2P, C] buffer, one BN batch each (the reference's two encoder
    calls): per-frame statistics, running stats updated frame a then frame b, and the
    downsample-residual apply with per-frame statistics of both BNs."""
    n, h, w = 2, 9, 11
    xa = (rnd((n, c, h, w), dt, 30) + 3.0).to(dt).double()
    xb = (rnd((n, c, h, w), dt, 31, scale=0.5) - 1.0).to(dt).double()
    da, db = rnd((n, c, h, w), dt, 32), rnd((n, c, h, w), dt, 33, scale=2.0)
    bn, bnd = _bn_mod(c, cuda, 34), _bn_mod(c, cuda, 35)
    rm, rv = bn.running_mean.double().cpu().clone(), bn.running_var.double().cpu().clone()
    cpu = lambda m: (m.weight.detach().double().cpu(), m.bias.detach().double().cpu())
    ya = F.batch_norm(xa, rm, rv, *cpu(bn), True, 0.1, 1e-5)
    yb = F.batch_norm(xb, rm, rv, *cpu(bn), True, 0.1, 1e-5)
    ra = F.batch_norm(da, None, None, *cpu(bnd), True, 0.1, 1e-5)
    rb = F.batch_norm(db, None, None, *cpu(bnd), True, 0.1, 1e-5)
    x = torch.cat([nhwc(xa), nhwc(xb)]).to(dt).to(cuda).contiguous()
    d = torch.cat([nhwc(da), nhwc(db)]).to(dt).to(cuda).contiguous()
    st = ops.bn_stats(x, bn, True, nseg=2)
    std = ops.bn_stats(d, bnd, True, nseg=2)
    y = ops.bn_apply(x, st, bn, act=1, xr=d, rstats=std, rbn=bnd, nseg=2)
    torch.cuda.synchronize()
    p = n * h * w
    close(nchw(y[:p], n, h, w), F.relu(ya + ra), dt)
    close(nchw(y[p:], n, h, w), F.relu(yb + rb), dt)
    close(bn.running_mean, rm, torch.float32, scale=1.0)
    close(bn.running_var, rv, torch.float32, scale=1.0)
    assert bn._cn_nbt == 2


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("pc", [(4 * 119 * 119, 64), (4 * 60 * 60, 1024)])
def test_batchnorm_stats_large(cuda, dt, pc):
    """Statistics at the step's sizes, with a channel mean far from zero (shifted sums)."""
    p, c = pc
    g = torch.Generator(device=cuda).manual_seed(36)
    off = torch.linspace(-20, 20, c, device=cuda)
    x = (torch.randn((p, c), generator=g, device=cuda) * 0.7 + off).to(dt)
    bn = _bn_mod(c, cuda, 37)
    mean, invstd = ops.bn_stats(x, bn, True)
    xd = x.double()
    m_ref = xd.mean(0)
    v_ref = xd.var(0, unbiased=False)
    torch.cuda.synchronize()
    assert (mean.double() - m_ref).abs().max().item() <= 1e-5 * (1 + m_ref.abs().max().item())
    assert ((invstd.double() - (v_ref + 1e-5).rsqrt()) / (v_ref + 1e-5).rsqrt()).abs().max().item() <= 1e-4


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_bn_eval(cuda, dt):
    n, c, h, w = 1, 256, 4, 6
    x = rnd((n, c, h, w), dt, 17)
    bn = _bn_mod(c, cuda, 18).eval()
    xg = nhwc(x).to(dt).to(cuda).contiguous()
    st = ops.bn_stats(xg, bn, False)
    y = ops.bn_apply(xg, st, bn, act=0)
    ref = F.batch_norm(x, bn.running_mean.double().cpu(), bn.running_var.double().cpu(),
                       bn.weight.detach().double().cpu(), bn.bias.detach().double().cpu(), False, 0.1, 1e-5)
    torch.cuda.synchronize()
    close(nchw(y, n, h, w), ref, dt)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("hw", [(237, 237), (49, 49), (12, 17)])
def test_maxpool_ceil(cuda, dt, hw):
    h, w = hw
    n, c = 2, 64
    x = rnd((n, c, h, w), dt, 19)
    xr = x.clone().requires_grad_(True)
    y = F.max_pool2d(xr, 3, 2, 1, ceil_mode=True)
    gy = rnd(y.shape, dt, 20)
    y.backward(gy)
    oh, ow = ops.pool_out(h), ops.pool_out(w)
    assert (oh, ow) == tuple(y.shape[2:])
    xg = nhwc(x).to(dt).to(cuda).contiguous()
    out = torch.empty((n * oh * ow, c), dtype=dt, device=cuda)
    am = torch.empty((n * oh * ow * c,), dtype=torch.uint8, device=cuda)
    nv.call("cn_maxpool_fwd", nv.dtype_code(dt), xg.data_ptr(), n, h, w, c, oh, ow, 3, 2, 1,
            out.data_ptr(), am.data_ptr(), nv.stream())
    gyg = nhwc(gy).to(dt).to(cuda).contiguous()
    dx = torch.empty_like(xg)
    nv.call("cn_maxpool_bwd", nv.dtype_code(dt), gyg.data_ptr(), am.data_ptr(), n, h, w, c, oh, ow,
            3, 2, 1, dx.data_ptr(), nv.stream())
    torch.cuda.synchronize()
    close(nchw(out, n, oh, ow), y.detach(), dt)
    close(nchw(dx, n, h, w), xr.grad, dt)


@pytest.mark.parametrize("hw", [((60, 60), (473, 473)), ((31, 41), (240, 320)), ((13, 13), (97, 97))])
def test_upsample_sigmoid(cuda, hw):
    (h, w), (H, W) = hw
    n = 2
    x = rnd((n, 1, h, w), torch.float32, 21, scale=3.0)
    xr = x.clone().requires_grad_(True)
    y = torch.sigmoid(F.interpolate(xr, size=(H, W), mode="bilinear", align_corners=False))
    gy = rnd(y.shape, torch.float32, 22)
    y.backward(gy)
    xg = x.float().to(cuda).contiguous()
    out = torch.empty((n, 1, H, W), dtype=torch.float32, device=cuda)
    nv.call("cn_upsample_sigmoid", xg.data_ptr(), n, h, w, H, W, 1, out.data_ptr(), nv.stream())
    din = torch.empty((n * h * w,), dtype=torch.float32, device=cuda)
    gyg = gy.float().to(cuda).contiguous()
    nv.call("cn_upsample_sigmoid_bwd", gyg.data_ptr(), out.data_ptr(), n, h, w, H, W, 1,
            din.data_ptr(), nv.stream())
    torch.cuda.synchronize()
    close(out, y.detach(), torch.float32)
    close(din.view(n, 1, h, w), xr.grad, torch.float32)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("bias", [False, True])
def test_gate_fwd_bwd(cuda, dt, bias):
    P, c = 333, 256
    z = rnd((P, c), dt, 23)
    v = rnd((P, c), dt, 24)
    g = rnd((1, c, 1, 1), torch.float32, 25, scale=0.1)
    gb = rnd((1,), torch.float32, 26) if bias else None
    zr, gr = z.clone().requires_grad_(True), g.clone().requires_grad_(True)
    gbr = gb.clone().requires_grad_(True) if bias else None
    m = torch.sigmoid(zr @ gr.view(c, 1) + (gbr if bias else 0))
    ref = torch.cat([zr * m, v], 1)
    gout = rnd(ref.shape, dt, 27)
    ref.backward(gout)
    from cosnet_amd.functions import GateCatFn
    zg = z.to(dt).to(cuda).requires_grad_(True)
    vg = v.to(dt).to(cuda)
    gg = g.float().to(cuda).requires_grad_(True)
    gbg = gb.float().to(cuda).requires_grad_(True) if bias else None
    out = GateCatFn.apply(zg, vg, gg, gbg, False)
    out.backward(gout.to(dt).to(cuda))
    torch.cuda.synchronize()
    close(out, ref.detach(), dt)
    close(zg.grad, zr.grad, dt)
    close(gg.grad, gr.grad, dt)
    if bias:
        close(gbg.grad, gbr.grad, dt)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_head_fwd_bwd(cuda, dt):
    P, c = 500, 256
    a, b = rnd((P, c), dt, 28), rnd((P, c), dt, 29)
    w = rnd((1, c, 1, 1), torch.float32, 30, scale=0.1)
    bias = rnd((1,), torch.float32, 31)
    ar, br, wr, biasr = (t.clone().requires_grad_(True) for t in (a, b, w, bias))
    ref = F.relu(ar + br) @ wr.view(c) + biasr
    gl = rnd((P,), torch.float32, 32)
    ref.backward(gl)
    from cosnet_amd.functions import HeadFn
    ag, bg = a.to(dt).to(cuda).requires_grad_(True), b.to(dt).to(cuda).requires_grad_(True)
    wg, bsg = w.float().to(cuda).requires_grad_(True), bias.float().to(cuda).requires_grad_(True)
    out = HeadFn.apply(ag, bg, wg, bsg, True)
    out.backward(gl.float().to(cuda))
    torch.cuda.synchronize()
    close(out, ref.detach(), dt)
    close(ag.grad, ar.grad, dt)
    close(bg.grad, br.grad, dt)
    close(wg.grad, wr.grad, dt)
    close(bsg.grad, biasr.grad, dt)


def test_loss_bce_l1(cuda):
    from cosnet_amd import loss as L
    g = torch.Generator().manual_seed(33)
    pred = torch.rand((2, 1, 37, 41), generator=g, dtype=torch.float64) * 0.98 + 0.01
    gt = (torch.rand((2, 1, 37, 41), generator=g) < 0.3).double()
    pr = pred.clone().requires_grad_(True)
    ratio = gt.numel() / float((gt >= 0.5).sum())
    ref = F.binary_cross_entropy(pr, gt, weight=torch.full_like(gt, ratio)) + 0.8 * F.l1_loss(pr, gt)
    ref.backward()
    pg = pred.float().to(cuda).requires_grad_(True)
    out = L.bce_l1(pg, gt.float().to(cuda))
    out.backward()
    torch.cuda.synchronize()
    assert abs(out.item() - ref.item()) <= 1e-5 * abs(ref.item())
    close(pg.grad, pr.grad, torch.float32)
    # device-count variant (no host sync) gives the same loss and gradient
    pg2 = pred.float().to(cuda).requires_grad_(True)
    out2 = L.bce_l1_device(pg2, gt.float().to(cuda))
    out2.backward()
    torch.cuda.synchronize()
    assert abs(out2.item() - ref.item()) <= 1e-5 * abs(ref.item())
    close(pg2.grad, pr.grad, torch.float32)
    # empty GT -> unweighted BCE (train.py:185-187)
    z = torch.zeros_like(gt)
    ref0 = F.binary_cross_entropy(pred, z) + 0.8 * F.l1_loss(pred, z)
    out0 = L.bce_l1(pred.float().to(cuda), z.float().to(cuda))
    assert abs(out0.item() - ref0.item()) <= 1e-5 * abs(ref0.item())
    out0d = L.bce_l1_device(pred.float().to(cuda), z.float().to(cuda))
    assert abs(out0d.item() - ref0.item()) <= 1e-5 * abs(ref0.item())


def test_sgd_step(cuda):
    from cosnet_amd.optim import SGD
    g = torch.Generator().manual_seed(34)
    ps = [torch.randn(s, generator=g) for s in [(64, 3, 7, 7), (256,), (10, 10)]]
    grads = [[torch.randn(p.shape, generator=g) for p in ps] for _ in range(3)]
    ref = [p.clone().requires_grad_(True) for p in ps]
    opt = torch.optim.SGD([{"params": ref[:1], "lr": 0.01}, {"params": ref[1:], "lr": 0.1}],
                          lr=0.01, momentum=0.9, weight_decay=5e-4)
    mine = [p.clone().to(cuda).requires_grad_(True) for p in ps]
    mopt = SGD([mine[:1], mine[1:]], [0.01, 0.1])
    for step in range(3):
        for p, gr in zip(ref, grads[step]):
            p.grad = gr.clone()
        for p, gr in zip(mine, grads[step]):
            p.grad = gr.clone().to(cuda)
        opt.step()
        mopt.step()
    torch.cuda.synchronize()
    for a, b in zip(mine, ref):
        assert torch.allclose(a.detach().cpu(), b.detach(), atol=1e-6, rtol=1e-5)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("dup", [False, True])
def test_sgd_refreshes_weight_copies(cuda, dt, dup):
    """cn_sgd updates the fp32 masters AND rewrites the compute-dtype GEMM copies (forward
    [Cout][KHW][Cp] and transposed [Cin][KHW][Cout]) in the same pass; the copies must equal a
    fresh preparation from the updated masters, and the masters torch.optim.SGD's for-loop
    semantics (duplicate entries updated once per occurrence)."""
    from cosnet_amd.optim import SGD
    g = torch.Generator().manual_seed(35)
    shapes = [((96, 64, 3, 3), None), ((70, 36, 1, 1), None), ((64, 3, 7, 7), 8),
              ((128, 256, 3, 3), None), ((256, 256), None), ((48,), None)]
    ps = [torch.randn(s, generator=g) * 0.05 for s, _ in shapes]
    ref = [p.clone().requires_grad_(True) for p in ps]
    mine = []
    for p in ps:
        q = p.clone().to(cuda)
        if q.dim() == 4:
            q = q.contiguous(memory_format=torch.channels_last)
        mine.append(torch.nn.Parameter(q))
    for (s, cp), q in zip(shapes, mine):  # cache entries exist before the first step
        if q.dim() >= 2:
            ops.WCACHE.get(q, dt, cin_pad=cp, need_t=cp is None)
    g0 = mine[:2] + (mine[:1] if dup else [])
    r0 = ref[:2] + (ref[:1] if dup else [])
    opt = torch.optim.SGD([{"params": r0, "lr": 0.01}, {"params": ref[2:], "lr": 0.1}],
                          lr=0.01, momentum=0.9, weight_decay=5e-4, foreach=False)
    mopt = SGD([g0, mine[2:]], [0.01, 0.1])
    for step in range(3):
        for p in ref:
            p.grad = torch.randn(p.shape, generator=g)
        for p, r in zip(mine, ref):
            p.grad = r.grad.clone().to(cuda)
            if p.dim() == 4:
                p.grad = p.grad.contiguous(memory_format=torch.channels_last)
        opt.step()
        mopt.step()
    torch.cuda.synchronize()
    for (s, cp), a, b in zip(shapes, mine, ref):
        assert torch.allclose(a.detach().cpu(), b.detach(), atol=1e-6, rtol=1e-5), s
        if a.dim() < 2:
            continue
        ents = ops.WCACHE.entries(a)
        assert len(ents) == 1 and ents[0][6][0] is not None, "entry must stay valid after the step"
        wf, wt = ents[0][0].clone(), ents[0][1]
        wt = wt.clone() if wt is not None else None
        ops.WeightCache.invalidate(ents[0][6])
        rf, rt = ops.WCACHE.get(a, dt, cin_pad=cp, need_t=cp is None)
        assert torch.equal(wf, rf), s
        if wt is not None:
            assert torch.equal(wt, rt), s


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("hw", [(13, 13), (15, 20), (31, 41)])
@pytest.mark.parametrize("both", [True, False])
def test_coattention_block(cuda, dt, hw, both):
    """CoattFn (linear + affinity bmm + row/col softmax + 2 gathers, fwd and bwd) against the
    oracle's restatement of rgbd_segmentation_RAA.py:150-170 in fp64.  S has std ~16 here
    (realistic, unscaled logits).  bf16 rounds V_a W^T and P to bf16 (SURVEY.md §7 iii), so
    its tolerance is J-level (0.15 of the output scale); fp32 is held to 2e-4."""
    from oracle.model_ref import RefModel
    from cosnet_amd.functions import CoattFn
    n, c = 2, 256
    h, w = hw
    va = rnd((n, c, h, w), dt, 40)
    vb = rnd((n, c, h, w), dt, 41)
    W = rnd((c, c), torch.float32, 42, scale=c ** -0.5)
    gza, gzb = rnd((n, c, h, w), dt, 43), rnd((n, c, h, w), dt, 44)
    var, wr = va.clone().requires_grad_(True), W.clone().requires_grad_(True)
    za, zb = RefModel.coattention(None, var, vb, wr)
    ((za * gza).sum() + ((zb * gzb).sum() if both else 0)).backward()
    vag = nhwc(va).to(dt).to(cuda).contiguous().requires_grad_(True)
    vbg = nhwc(vb).to(dt).to(cuda).contiguous()
    Wg = W.float().to(cuda).requires_grad_(True)
    ga, gb = CoattFn.apply(vag, vbg, Wg, (n, h * w))
    grads = [nhwc(gza).to(dt).to(cuda)]
    outs = [ga]
    if both:
        grads.append(nhwc(gzb).to(dt).to(cuda))
        outs.append(gb)
    torch.autograd.backward(outs, grads)
    torch.cuda.synchronize()
    tol = {torch.float32: 2e-4, torch.bfloat16: 0.15}[dt]
    for got, ref in ((ga, za), (gb, zb), (vag.grad, var.grad), (Wg.grad, wr.grad)):
        if got.dim() == 2 and got.shape[0] == n * h * w:
            got = nchw(got, n, h, w)
        got, ref = got.double().cpu(), ref.detach().double()
        err = (got - ref).abs().max().item() / ref.abs().max().item()
        assert err <= tol, (err, tol, tuple(ref.shape))


class _BN:
    """Minimal BatchNorm2d stand-in (the fields ops.* read)."""

    def __init__(self, c, cuda, seed):
        g = torch.Generator().manual_seed(seed)
        self.weight = (1 + 0.1 * torch.randn(c, generator=g)).to(cuda)
        self.bias = (0.1 * torch.randn(c, generator=g)).to(cuda)
        self.running_mean = torch.zeros(c, device=cuda)
        self.running_var = torch.ones(c, device=cuda)
        self.momentum, self.eps, self.affine = 0.1, 1e-5, True


FUSED_BN_CASES = [
    # n (per segment), cin, h, w, cout, k, stride, pad, dil, nseg  (rows straddle M tiles
    # and the segment boundary at non-multiples of 128; one case with > 2 tiles per segment)
    (2, 64, 13, 11, 128, 1, 1, 0, 1, 2),
    (2, 64, 13, 11, 64, 3, 1, 2, 2, 2),
    (1, 256, 30, 20, 256, 1, 1, 0, 1, 2),
    (2, 32, 15, 9, 512, 3, 1, 1, 1, 1),
    (2, 256, 7, 9, 128, 1, 2, 0, 1, 2),
    (4, 2048, 1, 1, 512, 1, 1, 0, 1, 2),   # the ASPP pooling branch (M = 2 x 4 rows)
]


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", FUSED_BN_CASES)
def test_conv_fwd_bn_epilogue_stats(cuda, dt, case):
    """cn_conv_fwd_bn: conv output + per-segment batch statistics from the GEMM epilogue against
    torch fp64 conv2d + batch_norm(training=True) per segment (running stats updated in segment
    order, unbiased running var)."""
    n, cin, h, w, cout, k, s, p, d, nseg = case
    x = rnd((nseg * n, cin, h, w), dt, 11, scale=2.0) + 3.0   # non-zero mean: shift exercised
    wt = rnd((cout, cin, k, k), dt, 12, scale=(2.0 / (cin * k * k)) ** 0.5)
    bias = rnd((cout,), torch.float32, 13, scale=0.5)
    ref = F.conv2d(x, wt, bias, s, p, d)
    bn = _BN(cout, cuda, 14)
    wf = wt.permute(0, 2, 3, 1).reshape(cout, k * k * cin).to(dt).to(cuda).contiguous()
    xg = nhwc(x).to(dt).to(cuda).contiguous()
    y, oh, ow, (mean, invstd) = ops.conv_fwd_bn(xg, nseg * n, h, w, wf, cout, k, s, p, d, bn, nseg,
                                                bias=bias.float().to(cuda))
    torch.cuda.synchronize()
    close(nchw(y, nseg * n, oh, ow), ref, dt)
    yr = nchw(y, nseg * n, oh, ow).double().cpu()   # statistics are of the values as stored
    rm, rv = torch.zeros(cout, dtype=torch.float64), torch.ones(cout, dtype=torch.float64)
    for sg in range(nseg):
        ys = yr[sg * n:(sg + 1) * n]
        mu = ys.mean(dim=(0, 2, 3))
        var = ys.var(dim=(0, 2, 3), unbiased=False)
        cnt = ys.numel() // cout
        assert torch.allclose(mean[sg * cout:(sg + 1) * cout].double().cpu(), mu, atol=1e-4 * (1 + mu.abs().max().item()), rtol=1e-5)
        assert torch.allclose(invstd[sg * cout:(sg + 1) * cout].double().cpu(), 1 / torch.sqrt(var + 1e-5), rtol=1e-4)
        rm = 0.9 * rm + 0.1 * mu
        rv = 0.9 * rv + 0.1 * var * cnt / (cnt - 1)
    assert torch.allclose(bn.running_mean.double().cpu(), rm, rtol=1e-4, atol=1e-5)
    assert torch.allclose(bn.running_var.double().cpu(), rv, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", [(2, 64, 13, 11, 128, 1, 0, 1), (2, 64, 13, 11, 64, 3, 2, 2),
                                  (4, 256, 30, 30, 64, 3, 1, 1), (1, 128, 9, 9, 256, 1, 0, 1)])
def test_conv_dgrad_bn_epilogue_reduce(cuda, dt, case):
    """cn_conv_dgrad_bn + cn_bn_bwd_apply: z = relu(bn(xpre)) (train mode) feeds conv(z, w);
    given dL/dconv_out, the fused dgrad returns dL/dz, dgamma, dbeta and bn_bwd_apply dL/dxpre --
    against torch fp64 autograd of the same graph."""
    n, cin, h, w, cout, k, p, d = case
    xpre = rnd((n, cin, h, w), dt, 21, scale=1.5) + 0.5
    wt = rnd((cout, cin, k, k), dt, 22, scale=(2.0 / (cin * k * k)) ** 0.5)
    gy = rnd((n, cout, h, w), dt, 23)
    bn = _BN(cin, cuda, 24)
    xr = xpre.clone().requires_grad_(True)
    gam = bn.weight.double().cpu().requires_grad_(True)
    bet = bn.bias.double().cpu().requires_grad_(True)
    z = F.relu(F.batch_norm(xr, None, None, gam, bet, True, 0.1, 1e-5))
    z.retain_grad()
    out = F.conv2d(z, wt, None, 1, p, d)
    out.backward(gy)
    xg = nhwc(xpre).to(dt).to(cuda).contiguous()
    mean, invstd = ops.bn_stats(xg, bn, True)
    wtt = wt.permute(1, 2, 3, 0).reshape(cin, k * k * cout).to(dt).to(cuda).contiguous()
    dz, dgam, dbet = ops.conv_dgrad_bn(nhwc(gy).to(dt).to(cuda).contiguous(), n, h, w, wtt, cin, k, p, d,
                                       xg, (mean, invstd), bn)
    dx = ops.bn_bwd_apply(xg, dz, (mean, invstd), bn, dgam, dbet)
    # the unfused HIP path on the same stored dy: dgrad, then the BN backward's own reduce + apply
    dz2 = ops.conv_dgrad(nhwc(gy).to(dt).to(cuda).contiguous(), n, h, w, wtt, cin, k, 1, p, d, h, w)
    dx2, dgam2, dbet2, _ = ops.bn_bwd(xg, dz2, None, (mean, invstd), bn, act=1)
    torch.cuda.synchronize()
    close(nchw(dz, n, h, w), z.grad, dt)
    assert torch.equal(dz, dz2)
    # fused == unfused up to the order of the fp32 sums (and one output rounding of dx)
    for a, b, t in ((dgam, dgam2, 1e-5), (dbet, dbet2, 1e-5),
                    (dx.float(), dx2.float(), 1e-5 if dt == torch.float32 else 8e-3)):
        assert ((a - b).abs().max() / b.abs().max()).item() <= t
    if dt == torch.float32:
        for got, ref in ((dgam, gam.grad), (dbet, bet.grad), (nchw(dx, n, h, w), xr.grad)):
            got, ref = got.double().cpu(), ref.double()
            assert (got - ref).abs().max().item() / ref.abs().max().item() <= 1e-4
    else:
        # bf16: the ReLU mask of a bf16-rounded pre-activation flips where bn(x) ~ 0, and one flip
        # is a full-size error in max-abs terms: dgamma max-rel, dx / dbeta mean-abs
        g, r = dgam.double().cpu(), gam.grad.double()
        assert (g - r).abs().max().item() / r.abs().max().item() <= 1e-2
        for got, ref in ((dbet, bet.grad), (nchw(dx, n, h, w), xr.grad)):
            got, ref = got.double().cpu(), ref.double()
            assert (got - ref).abs().mean().item() <= 2e-2 * ref.abs().mean().item()


def _dec_e4m3(u8):
    """Exact decode of OCP e4m3fn bytes (torch's float8_e4m3fn view)."""
    return u8.cpu().view(torch.float8_e4m3fn).double()


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_fp8_quant_matches_torch_e4m3fn(cuda, dt):
    """cn_fp8_quant (current scaling): scale = amax / 448, bytes = e4m3fn(x / scale) saturating,
    against torch's float8_e4m3fn conversion (round to nearest even)."""
    g = torch.Generator().manual_seed(3)
    x = (torch.randn((300, 96), generator=g) * 3.0).to(dt)
    st = ops.fp8_state(cuda)
    y8 = ops.fp8_quant(x.to(cuda), st, ops.FP8_CURRENT)
    torch.cuda.synchronize()
    amax = x.double().abs().max().item()
    assert abs(st[0].item() - amax / 448) <= 1e-6 * amax
    ref = (x.double() * st[1].double().cpu()).clamp(-448, 448).to(torch.float8_e4m3fn)
    got = _dec_e4m3(y8)
    diff = (got - ref.double()).abs()
    ulp = ref.double().abs().clamp_min(2 ** -6) * 2 ** -3   # one e4m3 mantissa step
    assert (diff <= ulp * 1.001).all()
    assert (diff == 0).double().mean().item() >= 0.999     # ties only may differ
    # delayed scaling: quantise with the stored scale, collect the amax, update
    y2 = ops.fp8_quant((x * 2).to(cuda), st, ops.FP8_DELAYED)
    ops.fp8_update(st)
    torch.cuda.synchronize()
    assert _dec_e4m3(y2).abs().max().item() == 448.0            # saturated at the old scale
    assert abs(st[0].item() - 2 * amax / 448) <= 1e-6 * amax      # next scale from the new amax


@pytest.mark.parametrize("case", [(2, 64, 13, 11, 128, 1, 1, 0, 1), (2, 32, 15, 9, 64, 3, 1, 2, 2),
                                  (1, 256, 12, 12, 256, 3, 1, 1, 1), (2, 256, 7, 9, 128, 1, 2, 0, 1),
                                  (4, 128, 30, 30, 512, 3, 1, 4, 4)])
def test_conv_fwd_fp8(cuda, case):
    """cn_conv_fwd_fp8 against fp64 conv2d of the exactly-decoded fp8 operands times their
    scales: checks the block-scaled MFMA's operand lane map (asymmetric data) and the
    dequantisation; only fp32 accumulation and the bf16 output rounding remain (1e-2)."""
    n, cin, h, w, cout, k, s, p, d = case
    x = rnd((n, cin, h, w), torch.float32, 31, scale=2.0)
    wt = rnd((cout, cin, k, k), torch.float32, 32, scale=(2.0 / (cin * k * k)) ** 0.5)
    xs, ws = ops.fp8_state(cuda), ops.fp8_state(cuda)
    x8 = ops.fp8_quant(nhwc(x).float().to(cuda).contiguous(), xs, ops.FP8_CURRENT)
    w8 = ops.fp8_quant(wt.permute(0, 2, 3, 1).reshape(cout * k * k, cin).float().to(cuda).contiguous(),
                       ws, ops.FP8_CURRENT).view(cout, k * k * cin)
    bias = rnd((cout,), torch.float32, 33).float().to(cuda)
    y, oh, ow = ops.conv_fwd_fp8(x8, n, h, w, w8, cout, k, s, p, d, xs, ws, bias=bias)
    torch.cuda.synchronize()
    xq = nchw(_dec_e4m3(x8), n, h, w) * xs[0].double().cpu()
    wq = _dec_e4m3(w8).reshape(cout, k, k, cin).permute(0, 3, 1, 2) * ws[0].double().cpu()
    ref = F.conv2d(xq, wq, bias.double().cpu(), s, p, d)
    got = nchw(y, n, oh, ow).double().cpu()
    err = ((got - ref).abs().max() / ref.abs().max()).item()
    assert err <= 1e-2, err


@pytest.mark.parametrize("case", [(2, 64, 13, 11, 128, 1, 1, 0, 1, 2), (2, 256, 17, 15, 256, 3, 1, 2, 2, 2),
                                  (1, 128, 30, 30, 512, 3, 1, 6, 6, 1), (2, 512, 9, 9, 64, 1, 1, 0, 1, 2)])
def test_conv_fwd_fp8_bn_epilogue_stats(cuda, case):
    """cn_conv_fwd_fp8_bn (configs[4]): the fp8 conv's output equals cn_conv_fwd_fp8's BITWISE
    (same kernel, EPI 1 only adds the reduction), and the per-segment batch statistics come out of
    the epilogue equal to fp64 statistics of that stored output (running stats in segment order)."""
    n, cin, h, w, cout, k, s, p, d, nseg = case
    x = rnd((nseg * n, cin, h, w), torch.float32, 41, scale=2.0) + 1.0
    wt = rnd((cout, cin, k, k), torch.float32, 42, scale=(2.0 / (cin * k * k)) ** 0.5)
    xs, ws = ops.fp8_state(cuda), ops.fp8_state(cuda)
    x8 = ops.fp8_quant(nhwc(x).float().to(cuda).contiguous(), xs, ops.FP8_CURRENT)
    w8 = ops.fp8_quant(wt.permute(0, 2, 3, 1).reshape(cout * k * k, cin).float().to(cuda).contiguous(),
                       ws, ops.FP8_CURRENT).view(cout, k * k * cin)
    bias = rnd((cout,), torch.float32, 43, scale=0.5).float().to(cuda)
    bn = _BN(cout, cuda, 44)
    y0, oh, ow = ops.conv_fwd_fp8(x8, nseg * n, h, w, w8, cout, k, s, p, d, xs, ws, bias=bias)
    y, oh, ow, (mean, invstd) = ops.conv_fwd_fp8_bn(x8, nseg * n, h, w, w8, cout, k, s, p, d, xs, ws,
                                                    bn, nseg, bias=bias)
    torch.cuda.synchronize()
    assert torch.equal(y, y0)
    yr = nchw(y, nseg * n, oh, ow).double().cpu()
    rm, rv = torch.zeros(cout, dtype=torch.float64), torch.ones(cout, dtype=torch.float64)
    for sg in range(nseg):
        ys = yr[sg * n:(sg + 1) * n]
        mu = ys.mean(dim=(0, 2, 3))
        var = ys.var(dim=(0, 2, 3), unbiased=False)
        cnt = ys.numel() // cout
        assert torch.allclose(mean[sg * cout:(sg + 1) * cout].double().cpu(), mu, atol=1e-4 * (1 + mu.abs().max().item()), rtol=1e-5)
        assert torch.allclose(invstd[sg * cout:(sg + 1) * cout].double().cpu(), 1 / torch.sqrt(var + 1e-5), rtol=1e-4)
        rm = 0.9 * rm + 0.1 * mu
        rv = 0.9 * rv + 0.1 * var * cnt / (cnt - 1)
    assert torch.allclose(bn.running_mean.double().cpu(), rm, rtol=1e-4, atol=1e-5)
    assert torch.allclose(bn.running_var.double().cpu(), rv, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", [(2, 256, 17, 15, 128, (1, 2, 5), 2), (1, 512, 30, 30, 512, (6, 12, 18), 1)])
def test_conv_fwd_bn_grouped_is_the_separate_launches(cuda, dt, case):
    """cn_conv_fwd_bn_grouped (the ASPP's atrous branches in one launch: per-problem weights,
    bias, dilation and statistics workspace) is BITWISE the G separate cn_conv_fwd_bn launches --
    outputs, batch statistics and running-stat updates -- and those are pinned to fp64 by
    test_conv_fwd_bn_epilogue_stats."""
    n, cin, h, w, cout, dils, nseg = case
    G = len(dils)
    x = rnd((nseg * n, cin, h, w), dt, 51, scale=2.0) + 1.0
    xg = nhwc(x).to(dt).to(cuda).contiguous()
    wfs, biases = [], []
    for g in range(G):
        wt = rnd((cout, cin, 3, 3), dt, 52 + g, scale=(2.0 / (cin * 9)) ** 0.5)
        wfs.append(wt.permute(0, 2, 3, 1).reshape(cout, 9 * cin).to(dt).to(cuda).contiguous())
        biases.append(rnd((cout,), torch.float32, 60 + g, scale=0.5).float().to(cuda))
    bns_a = [_BN(cout, cuda, 70 + g) for g in range(G)]
    bns_b = [_BN(cout, cuda, 70 + g) for g in range(G)]
    outs = ops.conv_fwd_bn_grouped(xg, nseg * n, h, w, wfs, cout, 3, list(dils), bns_a, nseg, biases=biases)
    refs = [ops.conv_fwd_bn(xg, nseg * n, h, w, wfs[g], cout, 3, 1, dils[g], dils[g], bns_b[g], nseg,
                            bias=biases[g]) for g in range(G)]
    torch.cuda.synchronize()
    for g in range(G):
        y, (m, i) = outs[g]
        yr, _, _, (mr, ir) = refs[g]
        assert torch.equal(y, yr), g
        assert torch.equal(m, mr) and torch.equal(i, ir), g
        assert torch.equal(bns_a[g].running_mean, bns_b[g].running_mean), g
        assert torch.equal(bns_a[g].running_var, bns_b[g].running_var), g


def _dec_e5m2(y8):
    return y8.cpu().view(torch.float8_e5m2).double()


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_fp8_quant_e5m2_matches_torch(cuda, dt):
    """cn_fp8_quant_fmt fmt 1 (the dgrad output gradients): scale = amax / 57344, bytes =
    e5m2(x / scale) saturating, against torch's float8_e5m2 conversion (round to nearest even)."""
    g = torch.Generator().manual_seed(4)
    x = (torch.randn((300, 96), generator=g) * 1e-3).to(dt)
    st = ops.fp8_state(cuda, ops.FP8_E5M2)
    y8 = ops.fp8_quant(x.to(cuda), st, ops.FP8_CURRENT, fmt=ops.FP8_E5M2)
    torch.cuda.synchronize()
    amax = x.double().abs().max().item()
    assert abs(st[0].item() - amax / 57344) <= 1e-6 * amax
    ref = (x.double() * st[1].double().cpu()).clamp(-57344, 57344).to(torch.float8_e5m2)
    got = _dec_e5m2(y8)
    diff = (got - ref.double()).abs()
    ulp = ref.double().abs().clamp_min(2 ** -14) * 2 ** -2   # one e5m2 mantissa step
    assert (diff <= ulp * 1.001).all()
    assert (diff == 0).double().mean().item() >= 0.999


@pytest.mark.parametrize("case", [(2, 256, 13, 11, 128, 3, 1, 1), (2, 128, 15, 9, 64, 1, 0, 1),
                                  (4, 512, 30, 30, 512, 3, 4, 4), (2, 256, 60, 60, 256, 3, 2, 2)])
@pytest.mark.parametrize("accumulate", [False, True])
def test_conv_dgrad_fp8(cuda, case, accumulate):
    """cn_conv_dgrad_fp8 (stride 1) against fp64 conv_transpose of the exactly-decoded e5m2 dY and
    e4m3 W^T times their scales: the A-format-e5m2 MFMA's operand map and the dequantisation; only
    fp32 accumulation and the bf16 output rounding remain (1e-2 of the output scale)."""
    n, cout, h, w, cin, k, p, d = case
    dy = rnd((n, cout, h, w), torch.float32, 41, scale=1e-2)
    wt = rnd((cout, cin, k, k), torch.float32, 42, scale=(2.0 / (cin * k * k)) ** 0.5)
    ds, ws = ops.fp8_state(cuda, ops.FP8_E5M2), ops.fp8_state(cuda)
    dy8 = ops.fp8_quant(nhwc(dy).float().to(cuda).contiguous(), ds, ops.FP8_CURRENT, fmt=ops.FP8_E5M2)
    # transposed weight [Cin][KH][KW][Cout] (the weight cache's dgrad copy)
    wT = wt.permute(1, 2, 3, 0).reshape(cin, k * k * cout).float().to(cuda).contiguous()
    w8 = ops.fp8_quant(wT, ws, ops.FP8_CURRENT)
    base = rnd((n, cin, h, w), torch.float32, 43)
    dx = nhwc(base).to(torch.bfloat16).to(cuda).contiguous()
    dx0 = dx.double().cpu()
    ops.conv_dgrad_fp8(dy8, n, h, w, w8, cin, k, p, d, h, w, ds, ws, out=dx, accumulate=accumulate)
    torch.cuda.synchronize()
    dyq = nchw(_dec_e5m2(dy8), n, h, w) * ds[0].double().cpu()
    wq = _dec_e4m3(w8).reshape(cin, k, k, cout).permute(3, 0, 1, 2) * ws[0].double().cpu()
    ref = F.conv_transpose2d(dyq, wq, None, 1, p, 0, 1, d)
    if accumulate:
        ref = ref + nchw(dx0, n, h, w)
    got = nchw(dx, n, h, w).double().cpu()
    err = ((got - ref).abs().max() / ref.abs().max()).item()
    assert err <= 1e-2, err


@pytest.mark.parametrize("case", [
    # n, cin, h, w, cout, k, stride, pad, dil  (cin, cout % 16; partial M, N and K tiles)
    (2, 256, 13, 11, 128, 3, 1, 2, 2),     # layer-3-like 3x3 dilated, split over K
    (2, 64, 30, 30, 256, 3, 1, 1, 1),      # many pixels: several K tiles per split
    (1, 512, 9, 9, 256, 3, 1, 1, 1),       # the ASPP bottleneck shape class
    (2, 128, 15, 9, 64, 1, 1, 0, 1),       # 1x1 (dense k-major B operand)
    (2, 96, 17, 19, 48, 3, 2, 1, 1),       # stride 2
])
@pytest.mark.parametrize("G", [1, 3])
def test_conv_wgrad_fp8(cuda, case, G):
    """cn_conv_wgrad_fp8 (configs[4] weight gradients: e5m2 dY x e4m3 X, both k-major, through
    the transposed byte reads ds_read_b64_tr_b8) against fp64 conv2d weight gradients of the
    exactly-decoded operands times their scales; G problems of one shape per launch, each with its
    own scales; deterministic (split-K slabs summed in a fixed order).  Only fp32 accumulation
    remains: 2e-3 of the output scale."""
    n, cin, h, w, cout, k, s, p, d = case
    oh, ow = ops.out_hw(h, w, k, s, p, d)
    jobs, refs = [], []
    for g in range(G):
        x = rnd((n, cin, h, w), torch.float32, 90 + g)
        gy = rnd((n, cout, oh, ow), torch.float32, 95 + g, scale=1e-2 * (g + 1))
        xs, ds = ops.fp8_state(cuda), ops.fp8_state(cuda, ops.FP8_E5M2)
        x8 = ops.fp8_quant(nhwc(x).float().to(cuda).contiguous(), xs, ops.FP8_CURRENT)
        dy8 = ops.fp8_quant(nhwc(gy).float().to(cuda).contiguous(), ds, ops.FP8_CURRENT, fmt=ops.FP8_E5M2)
        xq = nchw(_dec_e4m3(x8), n, h, w) * xs[0].double().cpu()
        gq = nchw(_dec_e5m2(dy8), n, oh, ow) * ds[0].double().cpu()
        wr = torch.zeros((cout, cin, k, k), dtype=torch.float64, requires_grad=True)
        F.conv2d(xq, wr, None, s, p, d).backward(gq)
        refs.append(wr.grad)
        dw = torch.full((cout, k * k * cin), float("nan"), dtype=torch.float32, device=cuda)
        jobs.append((x8, xs, dy8, ds, dw))
    ops.conv_wgrad_fp8(jobs, n, h, w, cin, oh, ow, cout, k, s, p, d)
    first = [j[4].clone() for j in jobs]
    ops.conv_wgrad_fp8(jobs, n, h, w, cin, oh, ow, cout, k, s, p, d)
    torch.cuda.synchronize()
    wp = torch.empty((cout, cin, k, k), device=cuda).contiguous(memory_format=torch.channels_last)
    for j, f, ref in zip(jobs, first, refs):
        got = ops.as_param_grad(j[4], wp).double().cpu()
        err = ((got - ref).abs().max() / ref.abs().max()).item()
        assert err <= 2e-3, err
        assert torch.equal(j[4], f)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("c", [3, 1])
def test_nchw_to_nhwc(cuda, dt, c):
    """cn_nchw_to_nhwc: the encoders' input frames (fp32 NCHW, rgbd_segmentation_RAA.py:143-148)
    to zero-padded 8-channel NHWC rows in the compute dtype -- exact."""
    n, h, w = 2, 37, 53
    x = torch.randn((n, c, h, w), generator=torch.Generator().manual_seed(11)).to(cuda)
    y = torch.full((n * h * w, 8), 7.0, dtype=dt, device=cuda)
    assert nv.call("cn_nchw_to_nhwc", nv.dtype_code(dt), x.data_ptr(), n, c, h, w, 8, y.data_ptr(),
                   nv.stream()) == 0
    ref = torch.zeros((n * h * w, 8), dtype=dt)
    ref[:, :c] = nhwc(x.cpu()).to(dt)
    assert torch.equal(y.cpu(), ref)
