import sys, torch
sys.path.insert(0, '.')
import torch.nn.functional as F
from cosnet_amd import ops, _native as nv
dev = torch.device('cuda:0')
for dt in (torch.float32, torch.bfloat16):
    n, c, h, w = 1, 8, 5, 5
    x = torch.randn(n, c, h, w, dtype=torch.float64).to(dt).double()
    xg = x.permute(0, 2, 3, 1).reshape(-1, c).to(dt).to(dev).contiguous()
    oh, ow = ops.pool_out(h), ops.pool_out(w)
    out = torch.zeros((n * oh * ow, c), dtype=dt, device=dev)
    am = torch.zeros((n * oh * ow * c,), dtype=torch.uint8, device=dev)
    nv.call("cn_maxpool_fwd", nv.dtype_code(dt), xg.data_ptr(), n, h, w, c, oh, ow, 3, 2, 1, out.data_ptr(), am.data_ptr(), nv.stream())
    torch.cuda.synchronize()
    ref = F.max_pool2d(x, 3, 2, 1, ceil_mode=True).permute(0, 2, 3, 1).reshape(-1, c)
    print(dt, 'maxpool err', (out.double().cpu() - ref).abs().max().item())
    print(out.cpu()[:3]); print(ref[:3])
    # cast copy
    y = torch.zeros_like(xg)
    ops.cast_copy(xg, y)
    torch.cuda.synchronize()
    print('cast err', (y - xg).abs().max().item())
    bn = torch.nn.BatchNorm2d(c).to(dev)
    st = ops.bn_stats(xg, bn, True)
    torch.cuda.synchronize()
    print('mean', st[0].cpu()[:4], x.mean(dim=(0, 2, 3))[:4])
    print('invstd', st[1].cpu()[:4], 1 / torch.sqrt(x.var(dim=(0, 2, 3), unbiased=False)[:4] + 1e-5))
