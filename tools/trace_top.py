"""Top (kernel, grid) groups by total time from a rocprofv3 kernel_trace.csv, per step.
usage: python tools/trace_top.py trace.csv steps [filter] [top]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2])
flt = sys.argv[3] if len(sys.argv) > 3 else ""
top = int(sys.argv[4]) if len(sys.argv) > 4 else 40
g = {}
for r in rows:
    n = r["Kernel_Name"]
    if flt not in n:
        continue
    key = (n[:70], r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    e = g.setdefault(key, [0, 0])
    e[0] += 1
    e[1] += d
tot = sum(v[1] for v in g.values())
print("total %.2f ms/step over %d groups" % (tot / 1e6 / steps, len(g)))
for k, (n, d) in sorted(g.items(), key=lambda kv: -kv[1][1])[:top]:
    print("%-70s %7sx%5sx%3s  n/step %5.1f  avg %7.1f us  %6.2f ms/step" % (k[0], k[1], k[2], k[3], n / steps, d / n / 1e3, d / 1e6 / steps))
