"""Time the co-attention block at the bench shape (B pairs, 60x60 features, C=256, bf16):
fused flash-style kernel vs the materialised-S path (affinity GEMM + softmax + 2 gathers).
Reports algorithmic TFLOP/s (3 x 2 HW^2 C per pair) and executed TFLOP/s
(4 x 2 HW^2 C: the fused kernel computes S once per direction)."""
import argparse
import json

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from cosnet_amd import ops
from cosnet_amd.functions import CoattFn

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=4)
ap.add_argument("--hw", type=int, default=3600)
ap.add_argument("--iters", type=int, default=20)
a = ap.parse_args()
dev = torch.device("cuda:0")
n, hw, c = a.n, a.hw, 256
g = torch.Generator().manual_seed(0)
va, vb, vat = [(torch.randn((n * hw, c), generator=g) * 0.7).to(torch.bfloat16).to(dev) for _ in range(3)]
W = (torch.randn((c, c), generator=g) * c ** -0.5).to(dev)
za = torch.empty((n * hw, c), dtype=torch.bfloat16, device=dev)
zb = torch.empty_like(za)


def timeit(fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / a.iters * 1e-3


alg = 3 * 2.0 * n * hw * hw * c
t_k = timeit(lambda: ops.coatt_fused(vat, va, vb, n, hw, za, zb))
t_8 = timeit(lambda: ops.coatt_f8(vat, va, vb, n, hw, za, zb))   # MX-fp8 (configs[4]), incl. prepass


def mat():
    with torch.no_grad():
        ops.COATT_FUSED = False
        CoattFn.apply(va, vb, W, (n, hw))
        ops.COATT_FUSED = True


def fused_block():
    with torch.no_grad():
        CoattFn.apply(va, vb, W, (n, hw))


t_m = timeit(mat)
t_f = timeit(fused_block)
print(json.dumps({"n": n, "hw": hw, "fused_kernel_us": t_k * 1e6,
                  "fused_kernel_alg_tflops": alg / t_k / 1e12,
                  "fused_kernel_exec_tflops": alg * 4 / 3 / t_k / 1e12,
                  "fp8_us": t_8 * 1e6, "fp8_alg_tflops": alg / t_8 / 1e12,
                  "block_fused_us": t_f * 1e6, "block_materialised_us": t_m * 1e6}))
