"""Loss trajectories of the fp8 training path (BASELINE configs[4]) against bf16 and fp32, over
several seeds: the distribution tests/test_gpu_fp8.py's bounds are set from.

    python tools/fp8_curve_dist.py [nseeds] [out.json]

For each seed base s: the same name-keyed weights, 4 SGD steps on the seeded batches s, s+1, ...
(97x97, B = 2 pairs, the eager step), in fp32, bf16 and fp8 (e4m3 forward convs, e5m2 dgrads and
3x3 weight gradients, MX-fp8 co-attention in inference and training since round 6).  Prints per-step relative loss gaps
fp8 vs bf16, fp8 vs fp32 and bf16 vs fp32 (the bf16 path's own floor on this chaotic
random-init network) and writes them as JSON.
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np
import torch

STEPS = 4


def trajectory(cuda, mode, seed0=100, graphed=False, size=97, batch=2, steps=STEPS):
    """Losses of `steps` SGD steps and the output-map means of a final eval forward."""
    import cosnet_amd as C
    from cosnet_amd.init_recipe import recipe_state_dict, synthetic_inputs
    from cosnet_amd.optim import SGD, reference_param_groups
    from cosnet_amd.train_step import TrainStep
    m = C.build_model(torch.float32 if mode == "fp32" else torch.bfloat16)
    m.load_state_dict(recipe_state_dict(m.state_dict()))
    m.encoder.main_classifier.requires_grad_(False)
    m = m.to(cuda).train()
    if mode == "fp8":
        m.set_fp8(True)
    g0, g1 = reference_param_groups(m)
    opt = SGD([g0, g1], [2.5e-6, 2.5e-3], momentum=0.9, weight_decay=5e-4)
    step = TrainStep(m, opt, batch, size, graphed=graphed)
    losses = []
    for i in range(steps):
        ins = [t.to(cuda) for t in synthetic_inputs(batch, size, size, seed=seed0 + i)]
        step.load(*ins)
        if graphed and i == 1:
            step.capture(warmup=0)     # record after one eager step (states, tables exist)
        loss = step([2.5e-6, 2.5e-3]) if (graphed and i >= 1) else step.eager([2.5e-6, 2.5e-3])
        losses.append(loss.item())
    with torch.no_grad():
        x1, x2, _ = m(*[t.to(cuda) for t in synthetic_inputs(batch, size, size, seed=999)[:4]])
    torch.cuda.synchronize()
    return np.array(losses), (x1.float().mean().item(), x2.float().mean().item()), m


def main():
    nseeds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    out = sys.argv[2] if len(sys.argv) > 2 else None
    cuda = torch.device("cuda:0")
    rows = []
    for k in range(nseeds):
        s0 = 100 + 100 * k
        r = {"seed0": s0}
        for mode in ("fp32", "bf16", "fp8"):
            l, mm, _ = trajectory(cuda, mode, s0)
            r[mode] = l.tolist()
            r[mode + "_map_means"] = mm
        f32, b16, f8 = (np.array(r[m]) for m in ("fp32", "bf16", "fp8"))
        r["gap_fp8_bf16"] = (np.abs(f8 - b16) / np.abs(b16)).tolist()
        r["gap_fp8_fp32"] = (np.abs(f8 - f32) / np.abs(f32)).tolist()
        r["gap_bf16_fp32"] = (np.abs(b16 - f32) / np.abs(f32)).tolist()
        r["mean_gap_fp8_bf16"] = abs(f8.mean() - b16.mean()) / b16.mean()
        rows.append(r)
        print("seed0 %d  fp8-bf16 %s (mean %.3f)  fp8-fp32 %s  bf16-fp32 %s" % (
            s0, np.round(r["gap_fp8_bf16"], 3), r["mean_gap_fp8_bf16"], np.round(r["gap_fp8_fp32"], 3),
            np.round(r["gap_bf16_fp32"], 3)), flush=True)
    allg = np.array([g for r in rows for g in r["gap_fp8_bf16"]])
    means = np.array([r["mean_gap_fp8_bf16"] for r in rows])
    summ = {"per_step_gap_fp8_bf16": {"median": float(np.median(allg)), "p90": float(np.quantile(allg, 0.9)),
                                      "max": float(allg.max())},
            "mean_gap_fp8_bf16": {"median": float(np.median(means)), "max": float(means.max())},
            "bf16_fp32_per_step_max": float(max(max(r["gap_bf16_fp32"]) for r in rows))}
    print(json.dumps(summ), flush=True)
    if out:
        with open(out, "w") as f:
            json.dump({"seeds": rows, "summary": summ, "steps": STEPS, "size": 97, "batch": 2}, f, indent=1)


if __name__ == "__main__":
    main()
