"""Do independent branches of a captured HIP graph run concurrently?  Two chains of under-filled
conv GEMMs (226 blocks each, the frame-batch layer-3 dgrad), captured (a) serialized on one
stream, (b) forked onto two streams; plus the same two variants eagerly.
usage: python tools/graph_concurrency.py"""
import sys

import torch

sys.path.insert(0, '.')
from cosnet_amd import ops  # noqa: E402

dev = torch.device('cuda:0')
dt = torch.bfloat16
L = 40


def chain(n=4, c=256, k=3, d=2):
    dy = torch.randn(n * 3600, c, device=dev).to(dt)
    wp = (torch.randn(c, c, k, k, device=dev) * 0.05).contiguous(memory_format=torch.channels_last)
    _, wt = ops.WCACHE.get(wp, dt)
    dx = torch.empty_like(dy)

    def run():
        for _ in range(L):
            ops.conv_dgrad(dy, n, 60, 60, wt, c, k, 1, d, d, 60, 60, out=dx)
    return run


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    a, b = chain(), chain()
    side = torch.cuda.Stream()
    main_s = torch.cuda.current_stream()

    def serial():
        a()
        b()

    def forked():
        side.wait_stream(torch.cuda.current_stream())
        a()
        with torch.cuda.stream(side):
            b()
        torch.cuda.current_stream().wait_stream(side)

    print("eager serial  %.3f ms" % timed(serial), flush=True)
    print("eager forked  %.3f ms" % timed(forked), flush=True)
    for name, fn in (("serial", serial), ("forked", forked)):
        s = torch.cuda.Stream()
        s.wait_stream(main_s)
        with torch.cuda.stream(s):
            fn()
        main_s.wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        print("graph %s  %.3f ms" % (name, timed(g.replay)), flush=True)
    print("(one chain = %d launches of a 226-block GEMM)" % L)


def two_graphs_main():
    """The same two chains captured as two single-stream graphs, replayed on two streams."""
    a, b = chain(), chain()
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    gs = []
    for fn, s in ((a, sa), (b, sb)):
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            fn()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            fn()
        gs.append(g)
    torch.cuda.synchronize()

    def rep():
        cur = torch.cuda.current_stream()
        sa.wait_stream(cur)
        sb.wait_stream(cur)
        with torch.cuda.stream(sa):
            gs[0].replay()
        with torch.cuda.stream(sb):
            gs[1].replay()
        cur.wait_stream(sa)
        cur.wait_stream(sb)
    print("two single-stream graphs  %.3f ms" % timed(rep), flush=True)


if __name__ == "__main__":
    main()
    two_graphs_main()
