"""Probe: which stream fork / join patterns inside one captured HIP graph does this ROCm accept?
(a weight-gradient side stream forked from the depth encoder's stream -- itself forked
from the capture origin -- ended in a segfault inside hipStreamEndCapture.)

Each case runs in its own subprocess (a segfault ends only that case) and prints OK / the error /
the signal.  Streams: O = capture origin, D = forked from O (the depth encoder), S = a side stream.

    python tools/probes/capture_fork_probe.py            # all cases
    python tools/probes/capture_fork_probe.py <case>     # one case (the child)
"""
import subprocess
import sys

CASES = {
    # S forked from D and joined back into D, D joined into O: the nested fork, properly joined
    "nested_joined": "fork(O,D); work(D); fork(D,S); work(S); join(S,D); work(D); join(D,O)",
    # S forked from D, joined straight into O (not into D)
    "nested_join_origin": "fork(O,D); work(D); fork(D,S); work(S); join(D,O); join(S,O)",
    # S forked from D and never joined (unjoined work at EndCapture)
    "nested_unjoined": "fork(O,D); work(D); fork(D,S); work(S); join(D,O)",
    # one side stream forked from O (RGB) and then from D (depth) in the same capture, joined into each
    "shared_side": "fork(O,D); fork(O,S); work(S); join(S,O); work(D); fork(D,S); work(S); join(S,D); join(D,O)",
    # the shared side stream, but its second use is joined into O only
    "shared_side_join_origin": "fork(O,D); fork(O,S); work(S); join(S,O); fork(D,S); work(S); join(S,O); join(D,O)",
    # allocation on S while capturing (the caching allocator's per-stream pools)
    "nested_alloc": "fork(O,D); fork(D,S); alloc(S); join(S,D); join(D,O)",
    # the side stream still capturing work after D was joined (S joined after D)
    "late_side": "fork(O,D); fork(D,S); join(D,O); work(S); join(S,O)",
}


def child(name):
    import torch
    dev = torch.device("cuda:0")
    st = {"O": torch.cuda.Stream(dev), "D": torch.cuda.Stream(dev), "S": torch.cuda.Stream(dev)}
    x = {k: torch.zeros(1 << 16, device=dev) for k in st}
    keep = []

    def fork(a, b):
        st[b].wait_stream(st[a])

    def join(a, b):
        st[b].wait_stream(st[a])

    def work(a):
        with torch.cuda.stream(st[a]):
            x[a].add_(1.0)

    def alloc(a):
        with torch.cuda.stream(st[a]):
            t = torch.empty(1 << 20, device=dev)
            t.fill_(1.0)
            keep.append(t)

    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=st["O"]):
        for stmt in CASES[name].split(";"):
            eval(stmt.strip(), {"fork": fork, "join": join, "work": work, "alloc": alloc,
                                "O": "O", "D": "D", "S": "S"})
    g.replay()
    torch.cuda.synchronize()
    print("OK", {k: float(v[0]) for k, v in x.items()})


def main():
    if len(sys.argv) > 1:
        return child(sys.argv[1])
    for name, prog in CASES.items():
        r = subprocess.run([sys.executable, __file__, name], capture_output=True, text=True, timeout=120)
        tail = (r.stdout.strip().splitlines() or [""])[-1]
        err = [l for l in r.stderr.splitlines() if "Error" in l or "error" in l or "Fatal" in l][-2:]
        print("%-26s rc=%-4d %-40s %s | %s" % (name, r.returncode, prog, tail, " / ".join(err)), flush=True)


if __name__ == "__main__":
    main()
