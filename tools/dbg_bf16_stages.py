"""bf16 vs fp32 HIP model, stage by stage, eval mode (473 calibration), one pair at 473^2."""
import sys
sys.path.insert(0, '.')
sys.path.insert(0, 'tests')
import torch
from conftest import golden
from test_gpu_configs import make_model
from cosnet_amd.init_recipe import synthetic_inputs

cuda = torch.device('cuda:0')
size = int(sys.argv[1]) if len(sys.argv) > 1 else 473
ra, rb, da, db, _, _ = synthetic_inputs(1, size, size, seed=5)
res = {}
for dt in (torch.float32, torch.bfloat16):
    m = make_model(cuda, dt, golden("bn_calibration_473.npz")).eval()
    st = {}
    with torch.no_grad():
        x1, x2, lab = m(ra.to(cuda), rb.to(cuda), da.to(cuda), db.to(cuda), stages=st)
    res[dt] = {k: v.float() for k, v in st.items() if torch.is_tensor(v)}
    res[dt].update(x1=x1.float(), x2=x2.float(), labels=lab.float())
a, b = res[torch.float32], res[torch.bfloat16]
for k in a:
    d = (a[k] - b[k]).abs()
    print("%-8s ref absmax %.3g  max|d| %.3g  mean|d| %.3g  rel %.3g" % (k, a[k].abs().max().item(), d.max().item(), d.mean().item(), d.mean().item() / a[k].abs().mean().item()))
    if k in ("x1", "x2", "labels"):
        print("         mask agree %.4f  mean32 %.4f mean16 %.4f" % (((a[k] > 0.5) == (b[k] > 0.5)).float().mean().item(), a[k].mean().item(), b[k].mean().item()))
