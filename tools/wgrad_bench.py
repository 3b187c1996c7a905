"""Per-launch time of the weight-gradient GEMM (split-K launch + fixed-order reduce) on the step's
conv shapes, operands cold in HBM (cycling > 600 MB of operand sets inside one recorded graph),
for each library given (COSNET_HIP_LIB is read at load, so each library runs in a child process).
usage: python tools/wgrad_bench.py [filter] [lib ...]"""
import os
import subprocess
import sys

# name, n (frames with gradient), cin, h, w, cout, k, stride, pad, dil
SHAPES = [
    ("l3_3x3_d2", 4, 256, 60, 60, 256, 3, 1, 2, 2),
    ("l4_3x3_d4", 4, 512, 60, 60, 512, 3, 1, 4, 4),
    ("aspp_3x3_d12", 4, 2048, 60, 60, 512, 3, 1, 12, 12),
    ("aspp_bneck_3x3", 4, 2560, 60, 60, 256, 3, 1, 1, 1),
    ("l2_3x3", 4, 128, 60, 60, 128, 3, 1, 1, 1),
    ("l2_3x3_s2", 4, 128, 119, 119, 128, 3, 2, 1, 1),
    ("l1_3x3", 4, 64, 119, 119, 64, 3, 1, 1, 1),
    ("l2_ds_1x1_s2", 4, 256, 119, 119, 512, 1, 2, 0, 1),
    ("stem_7x7_s2", 4, 8, 473, 473, 64, 7, 2, 3, 1),
    ("l3_1x1_1024to256", 4, 1024, 60, 60, 256, 1, 1, 0, 1),
    ("l3_1x1_256to1024", 4, 256, 60, 60, 1024, 1, 1, 0, 1),
    ("l4_1x1_2048to512", 4, 2048, 60, 60, 512, 1, 1, 0, 1),
    ("l4_1x1_512to2048", 4, 512, 60, 60, 2048, 1, 1, 0, 1),
]


def child(flt):
    import torch
    sys.path.insert(0, '.')
    from cosnet_amd import ops
    from cosnet_amd import _native as nv
    lib = nv.load()
    sys.path.insert(0, 'tools')
    from gemm_cold import gtime_sets
    dev = torch.device('cuda:0')
    dt = torch.bfloat16
    for (name, n, cin, h, w, cout, k, s, p, d) in SHAPES:
        if flt not in name:
            continue
        torch.manual_seed(0)
        oh = (h + 2 * p - d * (k - 1) - 1) // s + 1
        ow = (w + 2 * p - d * (k - 1) - 1) // s + 1
        fl = 2.0 * n * oh * ow * cout * k * k * cin
        sets, per = [], 0
        while per * len(sets) < 600e6 and len(sets) < 48:
            x = torch.randn(n * h * w, cin, device=dev).to(dt)
            dy = torch.randn(n * oh * ow, cout, device=dev).to(dt)
            dw = torch.empty((cout, k * k * cin), dtype=torch.float32, device=dev)
            sets.append(lambda x=x, dy=dy, dw=dw: ops.conv_wgrad(x, n, h, w, cin, dy, oh, ow, cout, k, s, p, d, dw=dw))
            per = (x.numel() + dy.numel()) * 2 + dw.numel() * 4
        splits = [int(v) for v in os.environ.get("WGRAD_SPLITS", "0").split(",")]
        # tiles of the plan's configuration (conv.hip wgrad_plan): 128x64 for N <= 64, 64x128 for
        # Cout <= 64, 128x128 otherwise; a target of s * tiles blocks makes the plan pick s splits
        nn = k * k * cin
        bm, bn = (128, 64) if nn <= 64 else ((64, 128) if cout <= 64 else (128, 128))
        tiles = -(-cout // bm) * -(-nn // bn)
        cfgs = [int(v) for v in os.environ.get("WGRAD_CFGS", "-1").split(",")]
        for sp, cf in [(a, b) for a in splits for b in cfgs]:
            lib.cn_gemm_force_config(cf)
            if sp:
                t = sp * tiles
                lib.cn_gemm_set_wgrad_target(t if t != 512 else 511)
            tw = gtime_sets(sets[:1], reps=20)
            tc = gtime_sets(sets)
            print("%-18s M=%5d N=%6d K=%6d s=%3s c=%3d | warm %7.1f us  cold %7.1f us  %6.0f TF/s (cold)" %
                  (name, cout, nn, n * oh * ow, sp or "auto", cf, tw * 1e6, tc * 1e6, fl / tc / 1e12), flush=True)
        lib.cn_gemm_set_wgrad_target(512)
        lib.cn_gemm_force_config(-1)
        del sets
        torch.cuda.empty_cache()


def main():
    if os.environ.get("WGRAD_CHILD"):
        child(os.environ.get("WGRAD_FILTER", ""))
        return
    flt = sys.argv[1] if len(sys.argv) > 1 and sys.argv[1] != "all" else ""
    libs = sys.argv[2:] or ["cosnet_amd/_lib/libcosnet_hip.so"]
    for lib in libs:
        print("## " + lib, flush=True)
        env = dict(os.environ, WGRAD_CHILD="1", WGRAD_FILTER=flt, COSNET_HIP_LIB=lib)
        rc = subprocess.run([sys.executable, __file__], env=env).returncode
        if rc:
            sys.exit(rc)


if __name__ == "__main__":
    main()
