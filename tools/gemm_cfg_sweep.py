"""Sweep the bf16 GEMM tile configurations (cn_gemm_force_config) over the step's conv shapes:
graph-timed TFLOP/s per config for fwd / dgrad / wgrad, and a correctness check of every
config against config 1 (the original 128x128 two-stage tile).
usage: python tools/gemm_cfg_sweep.py [filter] [configs, e.g. 1,2,3]"""
import sys

import torch

sys.path.insert(0, '.')
from cosnet_amd import _native as nv  # noqa: E402
from cosnet_amd import ops  # noqa: E402
from tools.bn_bench import gtime  # noqa: E402
from tools.gemm_lab import SHAPES  # noqa: E402

dev = torch.device('cuda:0')
dt = torch.bfloat16


def main():
    flt = sys.argv[1] if len(sys.argv) > 1 and sys.argv[1] != "all" else ""
    ncfg = nv.call("cn_gemm_force_config", -1) if False else int(nv.load().cn_gemm_force_config(-1))
    cfgs = [int(c) for c in sys.argv[2].split(",")] if len(sys.argv) > 2 else list(range(ncfg))
    best = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}
    base = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}
    for (name, n, cin, h, w, cout, k, s, p, d, cnt) in SHAPES:
        if flt not in name:
            continue
        torch.manual_seed(0)
        x = torch.randn(n * h * w, cin, device=dev).to(dt)
        wp = (torch.randn(cout, cin, k, k, device=dev) * 0.05).contiguous(memory_format=torch.channels_last)
        wf, wt = ops.WCACHE.get(wp, dt)
        oh, ow = ops.out_hw(h, w, k, s, p, d)
        nb = n // 2
        xb = x[:nb * h * w]
        dy = torch.randn(nb * oh * ow, cout, device=dev).to(dt)
        fl = 2.0 * n * oh * ow * cout * k * k * cin
        ref = {}
        line = "%-24s M=%7d N=%5d K=%6d" % (name, n * oh * ow, cout, k * k * cin)
        print(line, flush=True)
        for op in ("fwd", "dgrad", "wgrad"):
            if op == "dgrad" and (name == "stem7x7" or s != 1):
                continue
            res = []
            for c in cfgs:
                nv.load().cn_gemm_force_config(c)
                if op == "fwd":
                    y = torch.empty(n * oh * ow, cout, device=dev, dtype=dt)
                    f = (lambda y=y: ops.conv_fwd(x, n, h, w, wf, cout, k, s, p, d, out=y))
                    out, flops = y, fl
                elif op == "dgrad":
                    dx = torch.empty_like(xb)
                    f = (lambda dx=dx: ops.conv_dgrad(dy, nb, oh, ow, wt, cin, k, s, p, d, h, w, out=dx))
                    out, flops = dx, fl / 2
                else:
                    dw = torch.empty(cout, k * k * cin, device=dev)
                    f = (lambda dw=dw: ops.conv_wgrad(xb, nb, h, w, cin, dy, oh, ow, cout, k, s, p, d, dw=dw))
                    out, flops = dw, fl / 2
                t = gtime(f)
                f()
                torch.cuda.synchronize()
                if c == cfgs[0]:
                    ref[op] = out.float().clone()
                    err = 0.0
                else:
                    r = ref[op]
                    err = ((out.float() - r).abs().max() / r.abs().max().clamp_min(1e-20)).item()
                res.append((c, flops / t / 1e12, t, err))
            bt = min(r[2] for r in res)
            best[op] += bt * cnt / (1 if op == "fwd" else 2)
            b1 = [r for r in res if r[0] == 1]
            if b1:
                base[op] += b1[0][2] * cnt / (1 if op == "fwd" else 2)
            print("   %-5s " % op + " ".join("c%d:%5.0f%s" % (c, tf, "!" if e > 2e-2 else "") for c, tf, _, e in res),
                  flush=True)
    nv.load().cn_gemm_force_config(-1)
    print("weighted ms/step, config 1:", {k: round(v * 1e3, 2) for k, v in base.items()})
    print("weighted ms/step, best per shape:", {k: round(v * 1e3, 2) for k, v in best.items()})
    for sz in (4096, 8192):
        a = torch.randn(sz, sz, device=dev).to(dt)
        b = torch.randn(sz, sz, device=dev).to(dt)
        c_ = torch.empty(sz, sz, device=dev, dtype=dt)
        out = []
        for c in cfgs:
            nv.load().cn_gemm_force_config(c)
            tg = gtime(lambda: ops.gemm(a, b, sz, sz, sz, lda=sz, ldb=sz, out=c_, ldc=sz))
            out.append("c%d:%5.0f" % (c, 2.0 * sz ** 3 / tg / 1e12))
        nv.load().cn_gemm_force_config(-1)
        print("dense %d^3: %s" % (sz, " ".join(out)), flush=True)


if __name__ == "__main__":
    main()
