"""Variant-5 vs variant-1 training forward (with LSE) at a small map: which rows differ, and
whether the LSE (S / max / sum path) or only O (P.V path) is wrong (debug probe)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from cosnet_amd import _native as nv   # noqa: E402
from cosnet_amd import ops             # noqa: E402

dev = torch.device("cuda:0")
lib = nv.load()
for n, hw in ((1, 97), (1, 300)):
    g = torch.Generator().manual_seed(hw)
    vat, va, vb = [(torch.randn((n * hw, 256), generator=g) * 0.8).to(torch.bfloat16).to(dev) for _ in range(3)]
    res = {}
    for v in (1, 5):
        old = lib.cn_coatt_force_variant(v)
        za, zb = torch.empty_like(va), torch.empty_like(va)
        la = torch.empty((n, ops.hw_pad(hw)), dtype=torch.float32, device=dev)
        lb = torch.empty_like(la)
        ops.coatt_flash_fwd(vat, va, vb, n, hw, za, zb, la, lb)
        lib.cn_coatt_force_variant(old)
        torch.cuda.synchronize()
        res[v] = (za.float(), la[:, :hw].reshape(-1))
    dz = (res[1][0] - res[5][0]).abs().max(1).values
    dl = (res[1][1] - res[5][1]).abs()
    bad = (dz > 0.05).nonzero().flatten().tolist()
    print(n, hw, "bad O rows", bad[:20])
    print("   lse diff on bad rows", [round(dl[r].item(), 4) for r in bad[:20]])
    print("   lse diff max over all rows", dl.max().item())
    if bad:
        r = bad[0]
        print("   row", r, "O v1", res[1][0][r, :6].tolist(), "v5", res[5][0][r, :6].tolist())
        print("   lse v1", res[1][1][r].item(), "v5", res[5][1][r].item())
