"""Per-class GEMM time of the RECORDED step from a rocprofv3 --kernel-trace CSV (graph replays,
both encoder streams running as in the bench; no per-launch events).

    python tools/gemm_trace_shapes.py <run_kernel_trace.csv> [steps]

A class = (tile / loader / epilogue template, grid): the grid gives ceil(M/BM) x ceil(N/BN) x
batch*splits, the template the tile, so each class is one conv shape of the step.  Steps are
delimited by the SGD launch; the last `steps` complete steps are averaged.
"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    """T BMxBN wWMxWN sS L<LA><LB> e<EPI> p<PP> from the (mangled) template name."""
    m = re.search(r"gemm_kernelI(.*?)Li(\d+)E", name)
    if not m:
        return name[:60]
    t = "bf16" if m.group(1).startswith("DF16b") else ("f32" if m.group(1).startswith("f") else "f8")
    a = re.findall(r"Li(\d+)E", name[name.index("gemm_kernelI"):])
    a += ["0"] * (9 - len(a))
    return "%s %sx%s w%sx%s s%s L%s%s e%s p%s" % (t, a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7], a[8])


def main(path, nsteps=4):
    rows = [r for r in csv.DictReader(open(path)) if "spin_kernel" not in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    sgd = [i for i, r in enumerate(rows) if "sgd_k" in r["Kernel_Name"]]
    spans = list(zip(sgd[-nsteps - 1:-1], sgd[-nsteps:]))
    cls = defaultdict(lambda: [0, 0.0])
    tot_g = tot_all = 0.0
    for a, b in spans:
        for r in rows[a + 1:b + 1]:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            tot_all += d
            if "gemm_kernel" not in r["Kernel_Name"]:
                continue
            wg = int(r["Workgroup_Size_X"])
            grid = (int(r["Grid_Size_X"]) // wg, int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"]))
            k = (short(r["Kernel_Name"]), grid)
            cls[k][0] += 1
            cls[k][1] += d
            tot_g += d
    n = len(spans)
    print("steps %d: GEMM %.2f ms/step of %.2f ms/step serialized kernel time" % (n, tot_g / n / 1e3, tot_all / n / 1e3))
    print("%-44s %-16s %7s %9s %8s %6s" % ("template", "grid", "n/step", "ms/step", "us/launch", "%"))
    for (t, g), (c, d) in sorted(cls.items(), key=lambda kv: -kv[1][1]):
        print("%-44s %-16s %7.1f %9.3f %8.1f %6.2f" % (t, "x".join(map(str, g)), c / n, d / n / 1e3, d / c, 100 * d / tot_g))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 4)
