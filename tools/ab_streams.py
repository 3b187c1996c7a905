"""A/B of the step's stream layout on one box: graphed B=4 473x473 bf16 step with (a) one
stream, (b) depth encoder + depth head branch on a second stream (the shipped layout).
(A third layout, RGB weight gradients on a side stream of their own, measured 38.7 vs 34.0
ms/step -- slower -- and was dropped; profiles/r02_ab_streams.txt.)
usage: python tools/ab_streams.py [steps]"""
import sys
import time

import torch

sys.path.insert(0, '.')
import cosnet_amd as C  # noqa: E402
from cosnet_amd.init_recipe import recipe_state_dict, synthetic_inputs  # noqa: E402
from cosnet_amd.optim import SGD, reference_param_groups  # noqa: E402
from cosnet_amd.train_step import TrainStep  # noqa: E402

dev = torch.device('cuda:0')
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20


def run(conc, prio=0):
    torch.manual_seed(0)
    m = C.build_model(torch.bfloat16)
    m.load_state_dict(recipe_state_dict(m.state_dict()))
    m.encoder.main_classifier.requires_grad_(False)
    m = m.to(dev).train()
    m.concurrent_encoders = conc
    g0, g1 = reference_param_groups(m)
    opt = SGD([g0, g1], [1e-6, 1e-5])
    st = TrainStep(m, opt, 4, 473, graphed=True)
    if prio:
        st.stream = torch.cuda.Stream(device=dev, priority=prio)   # RGB / critical path
    st.load(*[t.to(dev) for t in synthetic_inputs(4, 473, 473, seed=1)])
    st.capture(warmup=2)
    for _ in range(3):
        st([1e-6, 1e-5])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        st([1e-6, 1e-5])
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    del st, m, opt
    torch.cuda.empty_cache()
    return dt


print("stream priority range", torch.cuda.Stream.priority_range())
for name, conc, prio in (("one stream", False, 0), ("two streams", True, 0),
                         ("two, main high", True, -1)) * 2:
    dt = run(conc, prio)
    print("%-16s %6.2f ms/step  %6.1f pairs/s" % (name, dt * 1e3, 4 / dt), flush=True)
