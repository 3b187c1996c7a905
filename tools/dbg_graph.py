"""Debug: per-parameter gradient agreement of a graph-replayed TrainStep vs two eager runs."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import cosnet_amd as C
from cosnet_amd.init_recipe import recipe_state_dict, synthetic_inputs
from cosnet_amd.optim import SGD, lr_poly, reference_param_groups
from cosnet_amd.train_step import TrainStep


def setup(dev, dtype, graphed, b=2, s=65):
    torch.manual_seed(0)
    m = C.build_model(dtype)
    m.load_state_dict(recipe_state_dict(m.state_dict()))
    m.encoder.main_classifier.requires_grad_(False)
    m = m.to(dev).train()
    g0, g1 = reference_param_groups(m)
    opt = SGD([g0, g1], [0.0, 0.0])
    st = TrainStep(m, opt, b, s, graphed=graphed)
    st.load(*[t.to(dev) for t in synthetic_inputs(b, s, s, seed=5)])
    return m, st


def lrs(i):
    lr = lr_poly(2.5e-4, i, 100, 0.9, 0)
    return [0.01 * lr, 10 * lr]


def main():
    dev = torch.device("cuda:0")
    dtype = torch.float32 if (len(sys.argv) < 2 or sys.argv[1] == "fp32") else torch.bfloat16
    warm = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    runs = [setup(dev, dtype, g) for g in (False, False, True)]
    for _, st in runs:
        st.opt.set_lrs(lrs(0))
        st.capture(warmup=warm)
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    for r in range(reps):
        losses = [float(st(lrs(warm + r))) for _, st in runs]
    torch.cuda.synchronize()
    print("losses", losses)
    names = {id(p): n for n, p in runs[0][0].named_parameters()}
    ps = [list(m.parameters()) for m, _ in runs]
    bad = 0
    for i, (a, b, g) in enumerate(zip(*ps)):
        if a.grad is None:
            if g.grad is not None:
                print("extra grad", names[id(a)])
            continue
        if g.grad is None:
            print("MISSING grad", i, names[id(a)])
            bad += 1
            continue
        sc = max(a.grad.abs().max().item(), 1e-20)
        ee = (a.grad - b.grad).abs().max().item() / sc
        eg = (a.grad - g.grad).abs().max().item() / sc
        pe = (a - b).abs().max().item()
        pg = (a - g).abs().max().item()
        flag = eg > max(4 * ee, 1e-4)
        if flag:
            bad += 1
        if flag or i % 40 == 0:
            print("%s %4d %-60s %-18s ee=%.3g eg=%.3g |p diff| ee=%.3g eg=%.3g sc=%.3g" % (
                "BAD" if flag else "ok ", i, names[id(a)], tuple(a.shape), ee, eg, pe, pg, sc))
    print("bad", bad)


if __name__ == "__main__":
    main()
