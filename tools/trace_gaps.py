"""Busy / idle structure of the graphed train step from a rocprofv3 --kernel-trace CSV.

    python tools/trace_gaps.py <run_kernel_trace.csv>

Steps are delimited by the SGD launch (one per step).  For each queue: kernel time, span and
the gaps between consecutive kernels on that queue; for the device: the union of busy time.
"""
import csv
import sys
from collections import defaultdict


def main(path):
    rows = list(csv.DictReader(open(path)))
    rows = [r for r in rows if "spin_kernel" not in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    sgd = [i for i, r in enumerate(rows) if "sgd_k" in r["Kernel_Name"]]
    print("steps (sgd launches):", len(sgd))
    for a, b in zip(sgd[-4:-1], sgd[-3:]):
        step = rows[a + 1:b + 1]
        t0 = int(step[0]["Start_Timestamp"]); t1 = int(step[-1]["End_Timestamp"])
        q = defaultdict(list)
        for r in step:
            q[r["Queue_Id"]].append(r)
        print(f"step span {(t1 - t0) / 1e6:.2f} ms, {len(step)} kernels")
        for qid, ks in sorted(q.items()):
            busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in ks) / 1e6
            gaps = [int(y["Start_Timestamp"]) - int(x["End_Timestamp"]) for x, y in zip(ks, ks[1:])]
            gpos = [g for g in gaps if g > 0]
            print(f"  queue {qid}: {len(ks)} kernels, busy {busy:.2f} ms, "
                  f"gaps>0 sum {sum(gpos) / 1e6:.2f} ms (median {sorted(gpos)[len(gpos) // 2] / 1e3 if gpos else 0:.1f} us), "
                  f"overlapping pairs {sum(1 for g in gaps if g <= 0)}")
        # device union
        iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in step)
        un = 0; cs, ce = iv[0]
        for s, e in iv[1:]:
            if s > ce:
                un += ce - cs; cs, ce = s, e
            else:
                ce = max(ce, e)
        un += ce - cs
        # idle before the step's first kernel, after the previous step's SGD (host issue gaps of
        # the program's graphs and host-issued kernels show up here)
        lead = t0 - int(rows[a]["End_Timestamp"])
        print(f"  device busy (union) {un / 1e6:.2f} ms, idle {(t1 - t0 - un) / 1e6:.2f} ms, "
              f"idle before the step {lead / 1e6:.3f} ms, period {(t1 - int(rows[a]['End_Timestamp'])) / 1e6:.2f} ms")


if __name__ == "__main__":
    main(sys.argv[1])
