"""Probe for horizontal fusion of the RGB and depth encoders (VERDICT r4 "next" #3).

Question: what does running one conv / BN of BOTH encoders as ONE launch of two problems buy over
the current two launches (one per encoder, the depth one on a second stream)?  For the layer-3
shapes of the configs[1] step (P = 2 x 4 x 60 x 60 = 28 800 rows: frames a and b, 4 pairs) it
times, per op, the device time of
  seq   -- the two launches back to back on one stream (no overlap at all),
  2str  -- the two launches on two streams, as the step runs them today (overlap where it fits),
  fused -- ONE launch covering both problems: the GEMM in its batched mode (blockIdx.z = problem,
           a_bs / b_bs / c_bs strides), the BN passes over the two problems' rows at once (2x the
           rows with twice the BN segments: the same bytes and block counts a two-problem BN
           kernel would have),
each as a chain of R launches recorded in a HIP graph and replayed (no host gaps), so
  per-op = (replay time) / R.  fused / seq < 2str / seq is what horizontal fusion would gain.
"""
import json
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from cosnet_amd import _native as nv   # noqa: E402
from cosnet_amd import ops             # noqa: E402

R = 40


def timed(fn, reps=3):
    """Median device ms of one replay of a graph holding R calls of fn (fn gets the call index)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for i in range(2):
            fn(i)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for i in range(R):
            fn(i)
    ts = []
    for _ in range(reps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts = sorted(ts[1:])
    return ts[len(ts) // 2] / R * 1e3   # us per call


def two_streams(f0, f1):
    """Call pattern of the step today: problem 0 on the current stream, problem 1 on a side stream
    forked / joined around each call pair (as the encoders' streams are joined at the head)."""
    side = torch.cuda.Stream()

    def fn(i):
        cur = torch.cuda.current_stream()
        side.wait_stream(cur)
        f0(i)
        with torch.cuda.stream(side):
            f1(i)
        cur.wait_stream(side)
    return fn


def two_streams_free(f0, f1):
    """Both problems' chains on two streams with no join between calls (the most overlap the two
    encoders could ever get)."""
    side = torch.cuda.Stream()
    state = {}

    def fn(i):
        cur = torch.cuda.current_stream()
        if i == 0:
            side.wait_stream(cur)
        f0(i)
        with torch.cuda.stream(side):
            f1(i)
        if i == R - 1 or i == 1:
            cur.wait_stream(side)
    return fn


def gemm_case(name, M, N, K, dev):
    bf = torch.bfloat16
    g = torch.Generator(device="cpu").manual_seed(1)
    A = (torch.randn((2, M, K), generator=g) * 0.1).to(bf).to(dev)
    B = (torch.randn((2, N, K), generator=g) * 0.1).to(bf).to(dev)
    C = torch.empty((2, M, N), dtype=bf, device=dev)

    def one(p):
        return lambda i: ops.gemm(A[p], B[p], M, N, K, lda=K, ldb=K, out=C[p], ldc=N)

    def fused(i):
        ops.gemm(A[0], B[0], M, N, K, lda=K, ldb=K, a_bs=M * K, b_bs=N * K, out=C[0], ldc=N,
                 c_bs=M * N, batch=2)
    f0, f1 = one(0), one(1)
    return {"op": name, "single": timed(f0),
            "seq": timed(lambda i: (f0(i), f1(i))),
            "2str": timed(two_streams(f0, f1)),
            "2str_free": timed(two_streams_free(f0, f1)),
            "fused": timed(fused)}


class _BN(torch.nn.BatchNorm2d):
    pass


def bn_case(name, P, C, dev, kind):
    bf = torch.bfloat16
    g = torch.Generator(device="cpu").manual_seed(2)
    x = torch.randn((2 * P, C), generator=g).to(bf).to(dev)
    r = torch.randn((2 * P, C), generator=g).to(bf).to(dev)
    bns = [_BN(C).to(dev) for _ in range(3)]
    st1 = ops.bn_stats(x[:P], bns[0], True, nseg=2)
    st2 = ops.bn_stats(x, bns[2], True, nseg=4)

    if kind == "apply":
        def one(p):
            return lambda i: ops.bn_apply(x[p * P:(p + 1) * P], st1, bns[p], act=1, res=r[p * P:(p + 1) * P], nseg=2)

        def fused(i):
            ops.bn_apply(x, st2, bns[2], act=1, res=r, nseg=4)
    else:
        def one(p):
            return lambda i: ops.bn_stats(x[p * P:(p + 1) * P], bns[p], True, nseg=2)

        def fused(i):
            ops.bn_stats(x, bns[2], True, nseg=4)
    f0, f1 = one(0), one(1)
    return {"op": name, "single": timed(f0),
            "seq": timed(lambda i: (f0(i), f1(i))),
            "2str": timed(two_streams(f0, f1)),
            "2str_free": timed(two_streams_free(f0, f1)),
            "fused": timed(fused)}


def main():
    dev = torch.device("cuda:0")
    P = 2 * 4 * 60 * 60
    rows = [
        gemm_case("gemm 1x1 1024->256 (M 28800, N 256, K 1024)", P, 256, 1024, dev),
        gemm_case("gemm 1x1 256->1024 (M 28800, N 1024, K 256)", P, 1024, 256, dev),
        gemm_case("gemm 3x3-sized K (M 28800, N 256, K 2304)", P, 256, 2304, dev),
        gemm_case("gemm layer-1 1x1 (M 2x4x119x119, N 64, K 256)", 2 * 4 * 119 * 119, 64, 256, dev),
        bn_case("bn_apply+res+relu [28800, 1024]", P, 1024, dev, "apply"),
        bn_case("bn_apply+res+relu [28800, 256]", P, 256, dev, "apply"),
        bn_case("bn_stats (+finalize) [28800, 256]", P, 256, dev, "stats"),
    ]
    for r in rows:
        r["fused_over_seq"] = r["fused"] / r["seq"]
        r["2str_over_seq"] = r["2str"] / r["seq"]
        print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)


if __name__ == "__main__":
    main()
