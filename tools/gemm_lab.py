"""Graph-timed per-shape throughput of the implicit-GEMM kernel on the step's conv shapes
(forward at the pair batch n=8, backward at n=4) plus plain dense GEMMs for reference.
usage: python tools/gemm_lab.py [filter]"""
import sys

import torch

sys.path.insert(0, '.')
from cosnet_amd import ops  # noqa: E402
from tools.bn_bench import gtime  # noqa: E402

dev = torch.device('cuda:0')
dt = torch.bfloat16
# name, n_fwd, cin, h, w, cout, k, stride, pad, dil, calls per step (fwd of both encoders)
SHAPES = [
    ("stem7x7", 8, 8, 473, 473, 64, 7, 2, 3, 1, 2),
    ("l1_1x1_256to64", 8, 256, 119, 119, 64, 1, 1, 0, 1, 4),
    ("l1_3x3_64", 8, 64, 119, 119, 64, 3, 1, 1, 1, 6),
    ("l1_1x1_64to256", 8, 64, 119, 119, 256, 1, 1, 0, 1, 8),
    ("l2_3x3_128", 8, 128, 60, 60, 128, 3, 1, 1, 1, 6),
    ("l2_1x1_512to128", 8, 512, 60, 60, 128, 1, 1, 0, 1, 6),
    ("l2_1x1_128to512", 8, 128, 60, 60, 512, 1, 1, 0, 1, 8),
    ("l3_1x1_1024to256", 8, 1024, 60, 60, 256, 1, 1, 0, 1, 27),
    ("l3_3x3_256_d2", 8, 256, 60, 60, 256, 3, 1, 2, 2, 29),
    ("l3_1x1_256to1024", 8, 256, 60, 60, 1024, 1, 1, 0, 1, 29),
    ("l4_1x1_2048to512", 8, 2048, 60, 60, 512, 1, 1, 0, 1, 4),
    ("l4_3x3_512_d4", 8, 512, 60, 60, 512, 3, 1, 4, 4, 6),
    ("l4_1x1_512to2048", 8, 512, 60, 60, 2048, 1, 1, 0, 1, 6),
    ("aspp_3x3_2048to512_d12", 8, 2048, 60, 60, 512, 3, 1, 12, 12, 6),
    ("aspp_bott_2560to256", 8, 2560, 60, 60, 256, 3, 1, 1, 1, 2),
]


def main():
    flt = sys.argv[1] if len(sys.argv) > 1 else ""
    tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}
    for (name, n, cin, h, w, cout, k, s, p, d, cnt) in SHAPES:
        if flt not in name:
            continue
        x = torch.randn(n * h * w, cin, device=dev).to(dt)
        wp = (torch.randn(cout, cin, k, k, device=dev) * 0.05).contiguous(memory_format=torch.channels_last)
        wf, wt = ops.WCACHE.get(wp, dt)
        y, oh, ow = ops.conv_fwd(x, n, h, w, wf, cout, k, s, p, d)
        fl = 2.0 * n * oh * ow * cout * k * k * cin
        tf = gtime(lambda: ops.conv_fwd(x, n, h, w, wf, cout, k, s, p, d, out=y))
        nb = n // 2
        xb, yb = x[:nb * h * w], y[:nb * oh * ow]
        dw = torch.zeros(cout, k * k * cin, device=dev)
        tw = gtime(lambda: ops.conv_wgrad(xb, nb, h, w, cin, yb, oh, ow, cout, k, s, p, d, dw=dw))
        res = "%-24s M=%7d N=%5d K=%6d  fwd %6.0f TF %7.1f us | wgrad %6.0f TF %7.1f us" % (
            name, n * oh * ow, cout, k * k * cin, fl / tf / 1e12, tf * 1e6, fl / 2 / tw / 1e12, tw * 1e6)
        tot["fwd"] += tf * cnt
        tot["wgrad"] += tw * cnt / 2
        if name != "stem7x7":
            dx = torch.empty_like(xb)
            td = gtime(lambda: ops.conv_dgrad(yb, nb, oh, ow, wt, cin, k, s, p, d, h, w, out=dx))
            res += " | dgrad %6.0f TF %7.1f us" % (fl / 2 / td / 1e12, td * 1e6)
            tot["dgrad"] += td * cnt / 2
        if k == 1 and s == 1:
            m_, n_, k_ = n * h * w, cout, cin
            a = x
            b = wf
            c = torch.empty(m_, n_, device=dev, dtype=dt)
            tg = gtime(lambda: ops.gemm(a, b, m_, n_, k_, lda=cin, ldb=cin, out=c, ldc=n_))
            res += " | dense %6.0f TF" % (2.0 * m_ * n_ * k_ / tg / 1e12)
            # the same products through torch (hipBLASLt): fwd x.W^T, wgrad dY^T.x, dgrad dY.W
            w2 = wf.view(cout, cin)
            t1 = gtime(lambda: torch.mm(a, w2.t(), out=c))
            dw2 = torch.empty(cout, cin, device=dev, dtype=dt)
            t2 = gtime(lambda: torch.mm(yb.t(), xb, out=dw2))
            dx2 = torch.empty_like(xb)
            t3 = gtime(lambda: torch.mm(yb, w2, out=dx2))
            res += " || hipBLASLt fwd %6.0f wgrad %6.0f dgrad %6.0f TF" % (
                fl / t1 / 1e12, fl / 2 / t2 / 1e12, fl / 2 / t3 / 1e12)
        print(res, flush=True)
    print("weighted ms/step (both encoders, pair fwd, frame-a bwd):", {k: round(v * 1e3, 2) for k, v in tot.items()})
    for sz in (4096, 8192):
        a = torch.randn(sz, sz, device=dev).to(dt)
        b = torch.randn(sz, sz, device=dev).to(dt)
        c = torch.empty(sz, sz, device=dev, dtype=dt)
        tg = gtime(lambda: ops.gemm(a, b, sz, sz, sz, lda=sz, ldb=sz, out=c, ldc=sz))
        tt = gtime(lambda: torch.mm(a, b.t(), out=c))
        print("dense %d^3: ours %6.0f TF, torch(hipBLASLt) %6.0f TF" % (sz, 2.0 * sz ** 3 / tg / 1e12, 2.0 * sz ** 3 / tt / 1e12), flush=True)


if __name__ == "__main__":
    main()
