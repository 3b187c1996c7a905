"""Peak device memory and time of one eager train step (bench config: 473x473, 4 pairs, bf16),
for the weight-gradient flush A/B (CN_WGRAD_FLUSH=end|layer, read at import: one process each).

    CN_WGRAD_FLUSH=layer python tools/mem_probe.py [batch] [size]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import cosnet_amd as C
from cosnet_amd import encoder_fn
from cosnet_amd.init_recipe import recipe_state_dict, synthetic_inputs
from cosnet_amd.optim import SGD, reference_param_groups
from cosnet_amd.train_step import TrainStep


def main():
    b = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    s = int(sys.argv[2]) if len(sys.argv) > 2 else 473
    dev = torch.device("cuda:0")
    m = C.build_model(torch.bfloat16)
    m.load_state_dict(recipe_state_dict(m.state_dict()))
    m.encoder.main_classifier.requires_grad_(False)
    m = m.to(dev).train()
    g0, g1 = reference_param_groups(m)
    opt = SGD([g0, g1], [1e-6, 1e-5], momentum=0.9, weight_decay=5e-4)
    st = TrainStep(m, opt, b, s, graphed=False)
    st.load(*[t.to(dev) for t in synthetic_inputs(b, s, s, seed=1234)])
    st.eager([1e-6, 1e-5])
    torch.cuda.synchronize()
    base = torch.cuda.memory_allocated()
    torch.cuda.reset_peak_memory_stats()
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        loss = st.eager([1e-6, 1e-5])
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    print(json.dumps({"wgrad_flush": encoder_fn.WGRAD_FLUSH, "batch": b, "size": s,
                      "resident_gb": base / 1e9, "peak_gb": torch.cuda.max_memory_allocated() / 1e9,
                      "eager_step_ms": sorted(ts)[1] * 1e3, "loss": float(loss.item())}), flush=True)


if __name__ == "__main__":
    main()
