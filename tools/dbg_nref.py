"""Diagnose bf16 N-reference parity: fused vs materialised co-attention vs the fp64 fixture."""
import sys
sys.path.insert(0, '.')
sys.path.insert(0, 'tests')
import numpy as np
import torch
from conftest import golden
from test_gpu_configs import make_model, _nref_inputs
from cosnet_amd import ops
from cosnet_amd.inference import multi_reference_x1

cuda = torch.device('cuda:0')
z = golden("nref5_473.npz")
t, td, rb, db = _nref_inputs(z)
ref = z["f64r/x1mean"].astype(np.float64)
rb16 = z["bf16/x1mean"].astype(np.float64)


def rep(name, g):
    g = g.double().cpu().numpy().reshape(ref.shape)
    print("%-28s agree %.4f mad %.4f mean %.4f" % (name, ((g > 0.5) == (ref > 0.5)).mean(), np.abs(g - ref).mean(), g.mean()))


print("ref bf16: agree %.4f mad %.4f" % (((rb16 > 0.5) == (ref > 0.5)).mean(), np.abs(rb16 - ref).mean()))
for dt in (torch.float32, torch.bfloat16):
    m = make_model(cuda, dt, golden("bn_calibration_473.npz")).eval()
    for fused in (True, False):
        ops.COATT_FUSED = fused
        g = multi_reference_x1(m, t.to(cuda), td.to(cuda), rb.to(cuda), db.to(cuda))
        rep("%s fused=%d nref" % (dt, fused), g)
    ops.COATT_FUSED = True
    with torch.no_grad():
        acc = 0
        for i in range(5):
            st = {}
            x1, _, _ = m(t.to(cuda), rb[i:i + 1].to(cuda), td.to(cuda), db[i:i + 1].to(cuda), stages=st)
            acc = acc + x1
            if i == 0:
                va = st["V_a"].float()
                print("  V_a absmax %.3g std %.3g" % (va.abs().max().item(), va.std().item()))
                W = m.rgb_similarity_weights.weight.float()
                vat = va @ W.t()
                S = vat @ st["V_b"].float().t()
                print("  S std %.3g absmax %.3g" % (S.std().item(), S.abs().max().item()))
        rep("%s loop fused" % dt, acc / 5)
