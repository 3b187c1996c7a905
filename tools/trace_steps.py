"""Per-step timeline analysis of a rocprofv3 kernel_trace.csv of bench.py (graph replays):
step boundaries are found from the first kernel of each replay (the input conversion
nchw_to_nhwc); for each step prints wall, union of busy intervals (any stream), the
serialized kernel sum and the idle time (gaps where no kernel runs).
usage: python tools/trace_steps.py trace.csv [first_kernel_substr]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
mark = sys.argv[2] if len(sys.argv) > 2 else "nchw_to_nhwc"
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Stream_Id"]) for r in rows)
starts = [i for i, e in enumerate(ev) if mark in e[2]]
# a step begins at every 4th input conversion (rgb_a, rgb_b, dep_a, dep_b)
starts = starts[::4]
print("steps found:", len(starts))
for si in range(len(starts) - 1):
    seg = ev[starts[si]:starts[si + 1]]
    t0, t1 = seg[0][0], seg[-1][1]
    busy, cur_s, cur_e = 0, None, None
    for s, e, _, _ in seg:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    ser = sum(e - s for s, e, _, _ in seg)
    streams = sorted(set(x[3] for x in seg))
    print("step %2d: %5d kernels  wall %6.2f ms  busy %6.2f ms  idle %5.2f ms  serial sum %6.2f ms  streams %s"
          % (si, len(seg), (t1 - t0) / 1e6, busy / 1e6, (t1 - t0 - busy) / 1e6, ser / 1e6, streams))
