"""Device memory of the recorded train step: one graph vs one-stream graphs per phase
(TrainStep split_graphs) vs the data-parallel chain at world 1 -- ADVICE r4: the split recording
uses one memory pool per stream, which cannot reuse each other's freed blocks.

    python tools/graph_mem_ab.py MODE [batch] [dtype]     MODE = one | split | chain, dtype bf16 | fp8

Prints one JSON line: memory allocated / reserved after recording + 3 replays, the peak over
warm-up, recording and replays, and the replay time per step.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import cosnet_amd as C
from cosnet_amd.init_recipe import recipe_state_dict, synthetic_inputs
from cosnet_amd.optim import SGD, reference_param_groups
from cosnet_amd.train_step import TrainStep


def main():
    mode = sys.argv[1]
    b = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    kind = sys.argv[3] if len(sys.argv) > 3 else "bf16"
    s = 473
    dev = torch.device("cuda:0")
    m = C.build_model(torch.bfloat16)
    m.load_state_dict(recipe_state_dict(m.state_dict()))
    if kind == "fp8":
        m.set_fp8(True)
    m.encoder.main_classifier.requires_grad_(False)
    m = m.to(dev).train()
    g0, g1 = reference_param_groups(m)
    opt = SGD([g0, g1], [1e-6, 1e-5], momentum=0.9, weight_decay=5e-4)
    st = TrainStep(m, opt, b, s, graphed=True, split_graphs=mode == "split", dp_chain=mode == "chain")
    st.load(*[t.to(dev) for t in synthetic_inputs(b, s, s, seed=1234)])
    torch.cuda.reset_peak_memory_stats()
    st.capture(warmup=1)
    lrs = [1e-6, 1e-5]
    st(lrs)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        st(lrs)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 3
    print(json.dumps({"mode": mode, "batch": b, "dtype": kind, "graphs": len([o for o in (st._rec or []) if o[0] == "graph"]) or 1,
                      "allocated_gb": torch.cuda.memory_allocated() / 1e9,
                      "reserved_gb": torch.cuda.memory_reserved() / 1e9,
                      "peak_allocated_gb": torch.cuda.max_memory_allocated() / 1e9,
                      "peak_reserved_gb": torch.cuda.max_memory_reserved() / 1e9,
                      "replay_ms": dt * 1e3}), flush=True)


if __name__ == "__main__":
    main()
