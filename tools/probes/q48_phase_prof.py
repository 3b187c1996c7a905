"""Per-phase shader-clock breakdown of the variant-5 co-attention loop (needs a library built with
-DQ48_PROF=1, loaded through COSNET_HIP_LIB).  Prints cycles per wave-tile for: DMA wait+barrier,
S-MFMA issue, softmax, PV (issue), and the clock-derived wave-tile time."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from cosnet_amd import _native as nv   # noqa: E402
from cosnet_amd import ops             # noqa: E402

dev = torch.device("cuda:0")
lib = nv.load()
buf = (ctypes.c_ulonglong * 8)()
for n, hw, mode in ((5, 3600, "nograd"), (4, 3600, "train")):
    g = torch.Generator().manual_seed(n)
    vat, va, vb = [(torch.randn((n * hw, 256), generator=g) * 0.7).to(torch.bfloat16).to(dev) for _ in range(3)]
    za, zb = torch.empty_like(va), torch.empty_like(va)
    la = torch.empty((n, ops.hw_pad(hw)), dtype=torch.float32, device=dev)
    lb = torch.empty_like(la)
    old = lib.cn_coatt_force_variant(5)
    fn = (lambda: ops.coatt_fused(vat, va, vb, n, hw, za, zb)) if mode == "nograd" else \
         (lambda: ops.coatt_flash_fwd(vat, va, vb, n, hw, za, zb, la, lb))
    fn(); torch.cuda.synchronize()
    lib.cn_q48_prof_read(buf)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        fn()
    e1.record()
    torch.cuda.synchronize()
    lib.cn_q48_prof_read(buf)
    lib.cn_coatt_force_variant(old)
    v = list(buf)
    tiles = max(v[4], 1)
    names = ["wait+barrier", "S issue", "softmax", "PV issue"]
    tot = sum(v[:4]) / tiles
    print(n, hw, mode, "kernel us %.1f" % (e0.elapsed_time(e1) / 10 * 1e3), "wave-tiles", tiles // 10,
          "cycles/wave-tile %.0f" % tot,
          " ".join("%s %.0f (%.0f%%)" % (nm, x / tiles, 100 * x / tiles / tot) for nm, x in zip(names, v[:4])))
    # whole-workgroup clocks vs the tile loop's (per wave: the 4 phases summed over a WG's 4 waves)
    nwg = int(nv.query("cn_coatt_q48_nwork", n, hw)) if hasattr(lib, "cn_coatt_q48_nwork") else 256
    wg = v[6] / 10 / nwg
    loop = sum(v[:4]) / 10 / nwg / 4
    print("   per workgroup: kernel clocks %.0f, tile loop %.0f (%.0f%%), merges %.0f (%.0f%%), rest %.0f" %
          (wg, loop, 100 * loop / wg, v[7] / 10 / nwg, 100 * v[7] / 10 / nwg / wg, wg - loop - v[7] / 10 / nwg))
