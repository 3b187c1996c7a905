"""Host-side cost of replaying a TWO-stream HIP graph (fork at the start, join at the end) vs a
one-stream graph vs two one-stream graphs on two streams joined by events outside the graphs.
Per-call host time without synchronisation, and the device time per replay; and, for the
two-stream graph, where the device idles (gaps between consecutive kernels of a replay,
measured with events after every 100 kernels is not possible inside a graph, so the total wall
time per replay is compared instead)."""
import time

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
    return ts, host, (time.perf_counter() - t0) * 1e3


def main(n=600, size=1 << 20):
    dev = torch.device("cuda:0")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    x = torch.zeros((size,), device=dev)
    y = torch.zeros((size,), device=dev)

    def branch(t, k):
        for _ in range(k):
            t.mul_(1.0001).add_(1.0)

    # one stream
    g1 = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s1):
        branch(x, 2); branch(y, 2)
    torch.cuda.synchronize()
    with torch.cuda.graph(g1, stream=s1):
        branch(x, n); branch(y, n)
    # two streams inside one graph: fork at the start, join at the end
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g2, stream=s1):
        cur = torch.cuda.current_stream()
        s2.wait_stream(cur)
        with torch.cuda.stream(s2):
            branch(y, n)
        branch(x, n)
        cur.wait_stream(s2)
    # two one-stream graphs on two streams, joined outside
    ga, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.graph(ga, stream=s1):
        branch(x, n)
    with torch.cuda.graph(gb, stream=s2):
        branch(y, n)
    torch.cuda.synchronize()

    def two_graphs():
        s2.wait_stream(s1)
        with torch.cuda.stream(s2):
            gb.replay()
        with torch.cuda.stream(s1):
            ga.replay()
        s1.wait_stream(s2)

    for name, fn in (("one-stream graph", lambda: g1.replay()), ("two-stream graph", lambda: g2.replay()),
                     ("two graphs, two streams", two_graphs)):
        fn(); fn()
        ts, host, wall = host_times(fn, 12)
        print("%-24s per-call host ms %s | 12 calls host %.1f ms, wall %.1f ms" %
              (name, [round(t, 2) for t in ts], host, wall), flush=True)


if __name__ == "__main__":
    main()
