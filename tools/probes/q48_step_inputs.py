"""The co-attention forward on the training step's own features (not random data): capture the
(vat, va, vb) the model hands ops.coatt_flash_fwd in one eager forward at the bench shape, then
time variant 1 vs variant 5 on them and (with a -DQ48_PROF=1 library) count the workgroups that
redo their key range because a row's logits outgrew the first tile's maximum by > Q48_GROWTH.
Also prints the logit statistics: max over keys minus first-tile max per row (log2 units)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import cosnet_amd as C                                         # noqa: E402
from cosnet_amd import _native as nv                           # noqa: E402
from cosnet_amd import ops                                     # noqa: E402
from cosnet_amd.init_recipe import recipe_state_dict, synthetic_inputs   # noqa: E402

dev = torch.device("cuda:0")
lib = nv.load()
m = C.build_model(torch.bfloat16)
m.load_state_dict(recipe_state_dict(m.state_dict()))
m = m.to(dev).train()
caps = []
real = ops.coatt_flash_fwd


def grab(vat, va, vb, n, hw, za, zb, la, lb):
    caps.append((vat.clone(), va.clone(), vb.clone(), n, hw, za is not None, zb is not None))
    return real(vat, va, vb, n, hw, za, zb, la, lb)


ops.coatt_flash_fwd = grab
x = [t.to(dev) for t in synthetic_inputs(4, 473, 473, seed=1234)]
out = m(x[0], x[1], x[2], x[3])
torch.cuda.synchronize()
ops.coatt_flash_fwd = real
prof = hasattr(lib, "cn_q48_prof_read")
buf = (ctypes.c_ulonglong * 6)()
L2E = 1.4426950408889634
for k, (vat, va, vb, n, hw, ha, hb) in enumerate(caps):
    q = vat.float().reshape(n, hw, -1)[:, :, :256]
    kk = vb.float().reshape(n, hw, -1)[:, :, :256]
    S = torch.bmm(q[:1], kk[:1].transpose(1, 2)) * L2E       # pair 0, direction 0
    g0 = (S.max(2).values - S[:, :, :32].max(2).values)
    print("call", k, "n", n, "hw", hw, "dirs", int(ha) + int(hb), "|S| max %.1f" % S.abs().max().item(),
          "growth over first tile (log2): median %.1f p99 %.1f max %.1f" % (
              g0.median().item(), g0.flatten().kthvalue(int(0.99 * g0.numel())).values.item(), g0.max().item()))
    za = torch.empty((n * hw, 256), dtype=torch.bfloat16, device=dev) if ha else None
    zb = torch.empty((n * hw, 256), dtype=torch.bfloat16, device=dev) if hb else None
    la = torch.empty((n, ops.hw_pad(hw)), dtype=torch.float32, device=dev)
    lb = torch.empty_like(la)
    for v in (1, 5):
        old = lib.cn_coatt_force_variant(v)
        real(vat, va, vb, n, hw, za, zb, la, lb)
        torch.cuda.synchronize()
        if prof:
            lib.cn_q48_prof_read(buf)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            real(vat, va, vb, n, hw, za, zb, la, lb)
        e1.record()
        torch.cuda.synchronize()
        redo = ""
        if prof:
            lib.cn_q48_prof_read(buf)
            redo = "redo workgroups per launch %.1f" % (buf[5] / 10)
        lib.cn_coatt_force_variant(old)
        print("   variant", v, "us %.1f" % (e0.elapsed_time(e1) / 10 * 1e3), redo)
