"""Probe: the train-mode forward of both encoders (no backward, no_grad) replayed as ONE
two-branch graph (RGB on the main stream, depth on a side stream) vs as TWO single-stream
graphs replayed concurrently on two streams (separate memory pools).  Measures whether the
per-node overhead of a multi-branch graph (profiles/r02_graph_launch_cost.txt) costs the step.
usage: python tools/graph_split_probe.py [batch] [size]"""
import sys

import torch

sys.path.insert(0, '.')
import cosnet_amd as C  # noqa: E402
from cosnet_amd.encoder_fn import encode_pair  # noqa: E402
from cosnet_amd.init_recipe import recipe_state_dict, synthetic_inputs  # noqa: E402

b = int(sys.argv[1]) if len(sys.argv) > 1 else 4
sz = int(sys.argv[2]) if len(sys.argv) > 2 else 473
dev = torch.device('cuda:0')
m = C.build_model(torch.bfloat16)
m.load_state_dict(recipe_state_dict(m.state_dict()))
m = m.to(dev).train()
m._set_dtype()
ra, rb, da, db, _, _ = [t.to(dev) for t in synthetic_inputs(b, sz, sz, seed=1)]
main = torch.cuda.Stream()
side = torch.cuda.Stream()


def both():
    cur = torch.cuda.current_stream()
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        d = encode_pair(m.depth_encoder, da, db)
    r = encode_pair(m.encoder, ra, rb)
    cur.wait_stream(side)
    return r, d


def timeit(fn, n=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


with torch.no_grad():
    # warm (weight caches, workspaces)
    with torch.cuda.stream(main):
        both()
    torch.cuda.synchronize()
    # A: one two-branch graph
    gA = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gA, stream=main):
        outA = both()
    tA = timeit(gA.replay)
    # B: two single-stream graphs, separate pools, replayed on two streams
    gR, gD = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.graph(gD, stream=side):
        outD = encode_pair(m.depth_encoder, da, db)
    with torch.cuda.graph(gR, stream=main):
        outR = encode_pair(m.encoder, ra, rb)

    def two():
        cur = torch.cuda.current_stream()
        main.wait_stream(cur)
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            gD.replay()
        with torch.cuda.stream(main):
            gR.replay()
        cur.wait_stream(main)
        cur.wait_stream(side)
    tB = timeit(two)
    tR = timeit(gR.replay)
    tD = timeit(gD.replay)
    # C: one single-stream graph of both (serial)
    gS = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gS, stream=main):
        encode_pair(m.depth_encoder, da, db)
        encode_pair(m.encoder, ra, rb)
    tS = timeit(gS.replay)
print("encoders fwd (b=%d, %d): two-branch graph %.2f ms | two single-stream graphs concurrently %.2f ms"
      " | RGB alone %.2f, depth alone %.2f, serial one-stream graph %.2f ms" % (b, sz, tA, tB, tR, tD, tS))
same = all(torch.equal(x, y) for x, y in zip(outA[0][:2], outR[:2]))
print("outputs identical:", same)
