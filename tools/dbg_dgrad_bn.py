import sys
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
import torch, torch.nn.functional as F
from test_gpu_kernels import rnd, nhwc, nchw, _BN
from cosnet_amd import ops
cuda = torch.device('cuda:0')
for dt in (torch.float32, torch.bfloat16):
    n, cin, h, w, cout, k, p, d = (4, 256, 30, 30, 64, 3, 1, 1)
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
    gyg = nhwc(gy).to(dt).to(cuda).contiguous()
    dz, dgam, dbet = ops.conv_dgrad_bn(gyg, n, h, w, wtt, cin, k, p, d, xg, (mean, invstd), bn)
    dx = ops.bn_bwd_apply(xg, dz, (mean, invstd), bn, dgam, dbet)
    dz2 = ops.conv_dgrad(gyg, n, h, w, wtt, cin, k, 1, p, d, h, w)
    dx2, dgam2, dbet2, _ = ops.bn_bwd(xg, dz2, None, (mean, invstd), bn, act=1)
    torch.cuda.synchronize()
    def e(a, b):
        a, b = a.double().cpu(), b.double()
        return (a - b).abs().max().item() / b.abs().max().item()
    print(dt, "dz", e(nchw(dz, n, h, w), z.grad), "dz==dz2", torch.equal(dz, dz2))
    print("  fused   dgam %.3g dbet %.3g dx %.3g" % (e(dgam, gam.grad), e(dbet, bet.grad), e(nchw(dx, n, h, w), xr.grad)))
    print("  unfused dgam %.3g dbet %.3g dx %.3g" % (e(dgam2, gam.grad), e(dbet2, bet.grad), e(nchw(dx2, n, h, w), xr.grad)))
    print("  fused vs unfused dgam %.3g dbet %.3g" % (e(dgam, dgam2.double().cpu()), e(dbet, dbet2.double().cpu())))
