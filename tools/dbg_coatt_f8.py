"""Debug probe of cn_coatt_f8_fwd: prepass images vs torch emulation, and the main kernel on
structured inputs."""
import math
import sys

import torch

sys.path.insert(0, '.')
from cosnet_amd import _native as nv  # noqa: E402
from cosnet_amd import ops  # noqa: E402

dev = torch.device('cuda:0')
n, hw, c = 1, 128, 256
g = torch.Generator().manual_seed(0)
vat, va, vb = [(torch.randn((n * hw, c), generator=g)).to(torch.bfloat16).to(dev) for _ in range(3)]
za = torch.empty((n * hw, c), dtype=torch.bfloat16, device=dev)
zb = torch.empty_like(za)
nws = int(nv.query("cn_coatt_f8_workspace_bytes", n, hw))
ws = torch.zeros((nws,), dtype=torch.uint8, device=dev)
nv.call("cn_coatt_f8_fwd", vat.data_ptr(), 256, va.data_ptr(), 256, vb.data_ptr(), 256, n, hw, c,
        za.data_ptr(), zb.data_ptr(), 256, None, None, ws.data_ptr(), nws, nv.stream())
torch.cuda.synchronize()
HWp = (hw + 63) // 64 * 64
nt = HWp // 64
rows = n * HWp
w = ws.cpu()
off = 0
a8 = w[off:off + rows * 256].view(rows, 256); off += rows * 256
b8 = w[off:off + rows * 256].view(rows, 256); off += rows * 256
as_ = w[off:off + rows * 8].view(rows, 8); off += rows * 8
bs = w[off:off + rows * 8].view(rows, 8); off += rows * 8
off = (off + 255) // 256 * 256
vtb = w[off:off + n * nt * 256 * 64].view(n, nt, 256, 64); off += n * nt * 256 * 64
vta = w[off:off + n * nt * 256 * 64].view(n, nt, 256, 64); off += n * nt * 256 * 64
vtbs = w[off:off + n * nt * 512].view(n, nt, 2, 32, 8)
dec = lambda u8: u8.contiguous().view(torch.float8_e4m3fn).double()
# rows: dequantise a8 with as_ (byte 4h + kk = block 2kk + h)
sc = torch.zeros(rows, 8, dtype=torch.float64)
for bi in range(8):
    sc[:, bi] = torch.exp2(as_[:, 4 * (bi & 1) + (bi >> 1)].double() - 127)
deq = (dec(a8).view(rows, 8, 32) * sc[..., None]).view(rows, 256)
x = vat.double().cpu()
print("rows: max |deq - x| / max|x| = %.3e" % ((deq[:hw] - x).abs().max() / x.abs().max()).item())
# V^T: dequantise vtb
vt = dec(vtb)[0]          # [nt, 256, 64]
vsc = vtbs[0].double()    # [nt, 2, 32, 8]
recon = torch.zeros(HWp, 256, dtype=torch.float64)
for t in range(nt):
    for h in range(2):
        for j in range(32):
            key = 64 * t + 32 * (j >> 4) + (j & 3) + 8 * ((j & 15) >> 2) + 4 * h
            for d in range(0, 256):
                s = math.ldexp(1.0, int(vsc[t, j >> 4, d & 31, d >> 5]) - 127)
                recon[key, d] = vt[t, d, 32 * h + j].item() * s
xb = vb.double().cpu()
print("vt: max |recon - v| / max|v| = %.3e" % ((recon[:hw] - xb).abs().max() / xb.abs().max()).item())
# main kernel output vs fp64 on the dequantised operands
qa, qb = deq[:hw], None
sc2 = torch.zeros(rows, 8, dtype=torch.float64)
for bi in range(8):
    sc2[:, bi] = torch.exp2(bs[:, 4 * (bi & 1) + (bi >> 1)].double() - 127)
qb = (dec(b8).view(rows, 8, 32) * sc2[..., None]).view(rows, 256)[:hw]
S = qa @ qb.T
ref = torch.softmax(S, dim=1) @ recon[:hw]
got = za.double().cpu()
print("Z_a: max err / max = %.3e" % ((got - ref).abs().max() / ref.abs().max()).item())
print("got[0,:8]", got[0, :8].tolist())
print("ref[0,:8]", ref[0, :8].tolist())
# structured: constant V -> Z must equal that constant
vc = torch.full((n * hw, c), 0.5, dtype=torch.bfloat16, device=dev)
nv.call("cn_coatt_f8_fwd", vat.data_ptr(), 256, vc.data_ptr(), 256, vc.data_ptr(), 256, n, hw, c,
        za.data_ptr(), zb.data_ptr(), 256, None, None, ws.data_ptr(), nws, nv.stream())
torch.cuda.synchronize()
print("const V: Z_a range", za.float().min().item(), za.float().max().item(), "(expect 0.5)")
