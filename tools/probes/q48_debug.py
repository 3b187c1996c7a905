"""Which rows / channels of the variant-5 co-attention differ from fp64 (debug probe)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from cosnet_amd import _native as nv   # noqa: E402
from cosnet_amd import ops             # noqa: E402

dev = torch.device("cuda:0")
lib = nv.load()
for n, hw in ((1, 97), (2, 63), (1, 300)):
    g = torch.Generator().manual_seed(hw)
    vat, va, vb = [(torch.randn((n * hw, 256), generator=g) * 0.8).to(torch.bfloat16).to(dev) for _ in range(3)]
    old = lib.cn_coatt_force_variant(5)
    za, zb = ops.coatt_fused(vat, va, vb, n, hw, torch.empty_like(va), torch.empty_like(va))
    lib.cn_coatt_force_variant(old)
    torch.cuda.synchronize()
    q = vat.double().reshape(n, hw, 256); b = vb.double().reshape(n, hw, 256)
    ra = (torch.softmax(q @ b.transpose(1, 2), 2) @ b).reshape(n * hw, 256)
    err = (za.double() - ra).abs()
    rows = err.max(1).values
    bad = (rows > 0.05).nonzero().flatten().tolist()
    print(n, hw, "bad rows", len(bad), bad[:40])
    if bad:
        r = bad[0]
        cols = (err[r] > 0.05).nonzero().flatten().tolist()
        print("   row", r, "bad cols", len(cols), cols[:64])
