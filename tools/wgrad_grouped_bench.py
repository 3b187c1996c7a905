"""Per-launch time of the grouped weight gradient (cn_conv_wgrad_grouped: G problems of one conv
shape, no split-K) on the step's groups, per tile configuration (cn_gemm_force_config; -1 = the
launch's own choice).  G distinct operand sets per launch (the layer-3 groups alone are 150-650 MB,
so every launch streams its operands from HBM as in the step).
usage: python tools/wgrad_grouped_bench.py [filter] [configs, e.g. -1,3,4,5]"""
import sys

import torch

sys.path.insert(0, '.')
sys.path.insert(0, 'tools')
from cosnet_amd import _native as nv  # noqa: E402
from cosnet_amd import ops  # noqa: E402
from gemm_cold import gtime_sets  # noqa: E402

dev = torch.device('cuda:0')
dt = torch.bfloat16
# name, G (identical convs of the RGB encoder), n (frames with gradient), cin, h, w, cout, k, stride, pad, dil
SHAPES = [
    ("l3_3x3_d2", 23, 4, 256, 60, 60, 256, 3, 1, 2, 2),
    ("l3_1x1_1024to256", 22, 4, 1024, 60, 60, 256, 1, 1, 0, 1),
    ("l3_1x1_256to1024", 23, 4, 256, 60, 60, 1024, 1, 1, 0, 1),
    ("l3_3x3_d2 depth", 6, 4, 256, 60, 60, 256, 3, 1, 2, 2),
    ("l3_1x1_1024to256 depth", 5, 4, 1024, 60, 60, 256, 1, 1, 0, 1),
    ("l3_1x1_256to1024 depth", 6, 4, 256, 60, 60, 1024, 1, 1, 0, 1),
    ("l4_1x1_2048to512", 2, 4, 2048, 60, 60, 512, 1, 1, 0, 1),
    ("l4_3x3_d4", 3, 4, 512, 60, 60, 512, 3, 1, 4, 4),
    ("l4_1x1_512to2048", 3, 4, 512, 60, 60, 2048, 1, 1, 0, 1),
    ("l2_3x3", 3, 4, 128, 60, 60, 128, 3, 1, 1, 1),
    ("l1_3x3", 3, 4, 64, 119, 119, 64, 3, 1, 1, 1),
]


def main():
    flt = sys.argv[1] if len(sys.argv) > 1 and sys.argv[1] != "all" else ""
    cfgs = [int(c) for c in sys.argv[2].split(",")] if len(sys.argv) > 2 else [-1, 3, 4, 5, 10, 11, 13, 15]
    lib = nv.load()
    for (name, G, n, cin, h, w, cout, k, s, p, d) in SHAPES:
        if flt not in name:
            continue
        G = min(G, ops.GROUP_MAX)
        torch.manual_seed(0)
        oh, ow = ops.out_hw(h, w, k, s, p, d)
        fl = 2.0 * n * oh * ow * cout * k * k * cin * G
        jobs = [(torch.randn(n * h * w, cin, device=dev).to(dt), torch.randn(n * oh * ow, cout, device=dev).to(dt),
                 torch.empty((cout, k * k * cin), dtype=torch.float32, device=dev)) for _ in range(G)]
        line = "%-18s G=%2d M=%5d N=%5d K=%6d |" % (name, G, cout, k * k * cin, n * oh * ow)
        for c in cfgs:
            lib.cn_gemm_force_config(c)
            t = gtime_sets([lambda: ops.conv_wgrad_grouped(jobs, n, h, w, cin, oh, ow, cout, k, s, p, d)], reps=5)
            line += " c%d %6.1f us %4.0f TF/s |" % (c, t * 1e6, fl / t / 1e12)
        lib.cn_gemm_force_config(-1)
        print(line, flush=True)
        del jobs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
