"""Per-kernel cost of a dependent chain of tiny kernels replayed as a HIP graph (the floor
every one of the step's ~1675 launches pays), one stream and two concurrent streams."""
import sys

import torch

sys.path.insert(0, '.')
from cosnet_amd import _native as nv  # noqa: E402

dev = torch.device('cuda:0')
x = torch.ones(64, device=dev)
y = torch.ones(64, device=dev)
N = 1000


def chain(t):
    for _ in range(N):
        nv.call("cn_scale", t.data_ptr(), 64, 1.0, nv.stream())


def run(fn):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 5 * 1e3 / N


side = torch.cuda.Stream()


def two():
    side.wait_stream(torch.cuda.current_stream())
    chain(x)
    with torch.cuda.stream(side):
        chain(y)
    torch.cuda.current_stream().wait_stream(side)


print("one stream: %.2f us per dependent tiny kernel" % run(lambda: chain(x)))
print("two streams (2 x %d kernels): %.2f us per kernel per stream" % (N, run(two)))


def two_graphs():
    """Each chain captured as its own single-stream graph; the two replayed on two streams."""
    ga, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    for g, t, s in ((ga, x, sa), (gb, y, sb)):
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            chain(t)
        torch.cuda.current_stream().wait_stream(s)
        with torch.cuda.graph(g, stream=s):
            chain(t)
    torch.cuda.synchronize()

    def rep():
        cur = torch.cuda.current_stream()
        sa.wait_stream(cur)
        sb.wait_stream(cur)
        with torch.cuda.stream(sa):
            ga.replay()
        with torch.cuda.stream(sb):
            gb.replay()
        cur.wait_stream(sa)
        cur.wait_stream(sb)
    rep()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        rep()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 5 * 1e3 / N


print("two single-stream graphs replayed concurrently: %.2f us per kernel per stream" % two_graphs())
