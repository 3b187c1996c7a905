"""Time ONE implicit-GEMM shape in isolation (for PMC passes over a single kernel).

    python tools/gemm_probe.py SHAPE [cfg] [reps]
SHAPE: aspp_fwd | aspp_wgrad | l3_fwd | l3_dgrad | l3_wgrad | l3_1x1 | dense8k
"""
import sys

import torch

sys.path.insert(0, '.')
from cosnet_amd import _native as nv  # noqa: E402
from cosnet_amd import ops  # noqa: E402

dev = torch.device('cuda:0')
dt = torch.bfloat16
CONV = {  # n, cin, h, w, cout, k, stride, pad, dil
    "aspp": (8, 2048, 60, 60, 512, 3, 1, 12, 12),
    "l3": (8, 256, 60, 60, 256, 3, 1, 2, 2),
    "l3_1x1": (8, 1024, 60, 60, 256, 1, 1, 0, 1),
    "l3b_1x1": (8, 256, 60, 60, 1024, 1, 1, 0, 1),
    "l4_1x1": (8, 2048, 60, 60, 512, 1, 1, 0, 1),
    "l4b_1x1": (8, 512, 60, 60, 2048, 1, 1, 0, 1),
    "l1_1x1": (8, 256, 119, 119, 64, 1, 1, 0, 1),
    "l1b_1x1": (8, 64, 119, 119, 256, 1, 1, 0, 1),
    "l2_1x1": (8, 512, 60, 60, 128, 1, 1, 0, 1),
    "l2b_1x1": (8, 128, 60, 60, 512, 1, 1, 0, 1),
    "asppb": (8, 2560, 60, 60, 256, 3, 1, 1, 1),
    "l3bd_1x1": (4, 256, 60, 60, 1024, 1, 1, 0, 1),
    "l3d_1x1": (4, 1024, 60, 60, 256, 1, 1, 0, 1),
    "l3d": (4, 256, 60, 60, 256, 3, 1, 2, 2),
    "l1w": (4, 64, 119, 119, 64, 3, 1, 1, 1),
    "l1w_1x1": (4, 256, 119, 119, 64, 1, 1, 0, 1),
    "l1wb_1x1": (4, 64, 119, 119, 256, 1, 1, 0, 1),
    "l2w_1x1": (4, 512, 60, 60, 128, 1, 1, 0, 1),
    "l2wb_1x1": (4, 128, 60, 60, 512, 1, 1, 0, 1),
    "l3w_1x1": (4, 1024, 60, 60, 256, 1, 1, 0, 1),
    "l3wb_1x1": (4, 256, 60, 60, 1024, 1, 1, 0, 1),
    "l3w": (4, 256, 60, 60, 256, 3, 1, 2, 2),
    "asppw": (4, 2048, 60, 60, 512, 3, 1, 12, 12),
    "l4": (8, 512, 60, 60, 512, 3, 1, 4, 4),
    "l1": (8, 64, 119, 119, 64, 3, 1, 1, 1),
    "l2": (8, 128, 60, 60, 128, 3, 1, 1, 1),
}


def main():
    name = sys.argv[1]
    cfg = int(sys.argv[2]) if len(sys.argv) > 2 else -1
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 50
    nv.load().cn_gemm_force_config(cfg)
    if len(sys.argv) > 4:
        nv.load().cn_gemm_set_wgrad_target(int(sys.argv[4]))
    if name == "affinity":  # S = Va_t Vb^T per pair, fp32 S (CoattFn.forward)
        nb, hw, c = 4, 3600, 256
        ldp = (hw + 7) // 8 * 8
        a = torch.randn(nb * hw, c, device=dev).to(dt)
        b = torch.randn(nb * hw, c, device=dev).to(dt)
        S = torch.empty((nb, hw, ldp), dtype=torch.float32, device=dev)
        fl = 2.0 * nb * hw * hw * c
        fn = lambda: ops.gemm(a, b, hw, hw, c, lda=c, ldb=c, a_bs=hw * c, b_bs=hw * c, out=S,  # noqa: E731
                              ldc=ldp, c_bs=hw * ldp, batch=nb)
    elif name == "dense8k":
        m = n = k = 8192
        a = torch.randn(m, k, device=dev).to(dt)
        b = torch.randn(n, k, device=dev).to(dt)
        c = torch.empty(m, n, device=dev, dtype=dt)
        fl = 2.0 * m * n * k
        fn = lambda: ops.gemm(a, b, m, n, k, lda=k, ldb=k, out=c, ldc=n)  # noqa: E731
    else:
        key, op = name.rsplit("_", 1)
        if op not in ("fwd", "dgrad", "wgrad"):
            key, op = name, "fwd"
        n, cin, h, w, cout, kk, s, p, d = CONV[key]
        x = torch.randn(n * h * w, cin, device=dev).to(dt)
        wp = (torch.randn(cout, cin, kk, kk, device=dev) * 0.05).contiguous(memory_format=torch.channels_last)
        wf, wt = ops.WCACHE.get(wp, dt)
        y, oh, ow = ops.conv_fwd(x, n, h, w, wf, cout, kk, s, p, d)
        fl = 2.0 * n * oh * ow * cout * kk * kk * cin
        dy = torch.randn_like(y)
        dx = torch.empty_like(x)
        dw = torch.zeros(cout, kk * kk * cin, device=dev)
        if op == "fwd":
            fn = lambda: ops.conv_fwd(x, n, h, w, wf, cout, kk, s, p, d, out=y)  # noqa: E731
        elif op == "dgrad":
            fn = lambda: ops.conv_dgrad(dy, n, oh, ow, wt, cin, kk, s, p, d, h, w, out=dx)  # noqa: E731
        else:
            fn = lambda: ops.conv_wgrad(x, n, h, w, cin, dy, oh, ow, cout, kk, s, p, d, dw=dw)  # noqa: E731
    fn()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / reps * 1e-3
    print("%s cfg %d: %.1f us  %.0f TFLOP/s" % (name, cfg, t * 1e6, fl / t / 1e12), flush=True)


if __name__ == "__main__":
    main()
