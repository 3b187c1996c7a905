"""Does re-launching a HIP graph wait for its previous launch?  Host-side time of each replay
call (no synchronisation between calls) for:
  A. a toy graph (a chain of N small kernels), one graph replayed back to back, and two
     identical graphs replayed alternately;
  B. the bench's recorded train step (TrainStep, 473x473, 4 pairs, bf16).
If a replay call returns in ~the host cost of submitting its nodes, the host runs ahead of the
GPU; if it takes ~the GPU time of one replay, each launch waits for the previous one, and the
GPU starts every replay with an empty queue (the idle gaps at the start of each step in the
kernel trace, profiles/r04_step_busy_final.txt).
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch


def host_times(fn, n):
    torch.cuda.synchronize()
    ts = []
    t0 = time.perf_counter()
    for _ in range(n):
        a = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - a) * 1e3)
    host = (time.perf_counter() - t0) * 1e3
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e3
    return ts, host, wall


def toy(n_kernels=1500):
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream()
    x = torch.zeros((1 << 16,), device=dev)
    graphs = []
    for _ in range(2):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            for _ in range(3):
                x.add_(1.0)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            for _ in range(n_kernels):
                x.add_(1.0)
        graphs.append(g)
    for g in graphs:
        g.replay()
    torch.cuda.synchronize()
    ts, host, wall = host_times(lambda: graphs[0].replay(), 20)
    print("toy one graph : per-call host ms %s ... | 20 calls host %.2f ms, wall %.2f ms" %
          ([round(t, 2) for t in ts[:6]], host, wall), flush=True)
    k = [0]

    def alt():
        graphs[k[0] & 1].replay()
        k[0] += 1
    ts, host, wall = host_times(alt, 20)
    print("toy alternate : per-call host ms %s ... | 20 calls host %.2f ms, wall %.2f ms" %
          ([round(t, 2) for t in ts[:6]], host, wall), flush=True)


def step():
    import cosnet_amd as C
    from cosnet_amd.init_recipe import recipe_state_dict, synthetic_inputs
    from cosnet_amd.optim import SGD, reference_param_groups
    from cosnet_amd.train_step import TrainStep
    dev = torch.device("cuda:0")
    m = C.build_model(torch.bfloat16)
    m.load_state_dict(recipe_state_dict(m.state_dict()))
    m.encoder.main_classifier.requires_grad_(False)
    m = m.to(dev).train()
    g0, g1 = reference_param_groups(m)
    opt = SGD([g0, g1], [0.0, 0.0], momentum=0.9, weight_decay=5e-4)
    st = TrainStep(m, opt, 4, 473, graphed=True)
    st.load(*[t.to(dev) for t in synthetic_inputs(4, 473, 473, seed=1234)])
    st.capture(warmup=2)
    for _ in range(3):
        st([1e-6, 1e-5])
    ts, host, wall = host_times(lambda: st([1e-6, 1e-5]), 10)
    print("train step    : per-call host ms %s | 10 calls host %.2f ms, wall %.2f ms" %
          ([round(t, 2) for t in ts], host, wall), flush=True)
    print("  (concurrent encoders %s)" % m.concurrent_encoders)


if __name__ == "__main__":
    if os.environ.get("PROBE_TOY", "1") == "1":
        toy()
    step()
