"""Where the graphed train step's time goes between the two encoder streams: time the same step
(473x473, 4 pairs, bf16, recorded graph) for models whose RGB / depth encoders have different
numbers of bottleneck blocks.  If shrinking the depth encoder (second stream) does not shorten
the step, its work is hidden behind the RGB chain; the step time per layer-3 block of the RGB
encoder is the marginal cost of the critical path.  Timing probe only (not the metric).
usage: python tools/critical_path_probe.py"""
import sys
import time

import torch

sys.path.insert(0, '.')
from cosnet_amd import Bottleneck, RGBDSegmentation_RAA  # noqa: E402
from cosnet_amd.init_recipe import recipe_state_dict, synthetic_inputs  # noqa: E402
from cosnet_amd.optim import SGD, reference_param_groups  # noqa: E402
from cosnet_amd.train_step import TrainStep  # noqa: E402

CASES = [("rgb[3,4,23,3] depth[3,4,6,3] (the model)", [3, 4, 23, 3], [3, 4, 6, 3]),
         ("rgb[3,4,23,3] depth[1,1,1,1]", [3, 4, 23, 3], [1, 1, 1, 1]),
         ("rgb[3,4,12,3] depth[3,4,6,3]", [3, 4, 12, 3], [3, 4, 6, 3]),
         ("rgb[3,4,6,3]  depth[3,4,6,3]", [3, 4, 6, 3], [3, 4, 6, 3]),
         ("rgb[3,4,6,3]  depth[1,1,1,1]", [3, 4, 6, 3], [1, 1, 1, 1])]


def run(rgb, dep, steps=15):
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    m = RGBDSegmentation_RAA(Bottleneck, rgb, dep, num_classes=1)
    m.set_compute_dtype(torch.bfloat16)
    m.load_state_dict(recipe_state_dict(m.state_dict()))
    m.encoder.main_classifier.requires_grad_(False)
    m = m.to(dev).train()
    g0, g1 = reference_param_groups(m)
    opt = SGD([g0, g1], [1e-6, 1e-5], momentum=0.9, weight_decay=5e-4)
    step = TrainStep(m, opt, 4, 473, graphed=True)
    step.load(*[t.to(dev) for t in synthetic_inputs(4, 473, 473, seed=1)])
    step.capture(warmup=2)
    for _ in range(3):
        step([1e-6, 1e-5])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step([1e-6, 1e-5])
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def main():
    for name, rgb, dep in CASES:
        ms = run(rgb, dep)
        print("%-44s %7.2f ms/step" % (name, ms), flush=True)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
