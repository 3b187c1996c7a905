"""Which torch ops still launch device kernels / copies inside one eager training step?

    python tools/copy_audit.py
Prints the aten ops of one eager bench step (after warmup) that run on the GPU, with shapes,
so stray copies / fills on the hot path can be found.  Development tool.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from torch.profiler import ProfilerActivity, profile

import cosnet_amd as C
from cosnet_amd.init_recipe import recipe_state_dict, synthetic_inputs
from cosnet_amd.optim import SGD, reference_param_groups
from cosnet_amd.train_step import TrainStep


def main():
    dev = torch.device("cuda:0")
    m = C.build_model(torch.bfloat16)
    m.load_state_dict(recipe_state_dict(m.state_dict()))
    m.encoder.main_classifier.requires_grad_(False)
    m = m.to(dev).train()
    g0, g1 = reference_param_groups(m)
    opt = SGD([g0, g1], [1e-6, 1e-5])
    st = TrainStep(m, opt, 4, 473, graphed=False)
    st.load(*[t.to(dev) for t in synthetic_inputs(4, 473, 473, seed=1)])
    st.capture(warmup=2)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        st.eager([1e-6, 1e-5])
        torch.cuda.synchronize()
    keys = prof.key_averages(group_by_input_shape=True)
    rows = []
    for k in keys:
        if k.key.startswith("aten::") and k.device_time_total > 0:
            rows.append((k.device_time_total, k.count, k.key, str(k.input_shapes)[:120]))
    rows.sort(reverse=True)
    for t, n, key, shp in rows[:40]:
        print("%9.1f us %4d  %-28s %s" % (t, n, key, shp))


if __name__ == "__main__":
    main()
