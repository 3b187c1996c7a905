"""Summarise rocprofv3 PMC passes into per-kernel-family HBM traffic per launch.

    python tools/pmc_summary.py [--steps 2] FETCH_DIR WRITE_DIR [MFMA_DIR] > profiles/rNN_pmc_step_traffic.json

Each *_DIR holds the `*_counter_collection.csv` of ONE `rocprofv3 --pmc` pass over the same
command (`python bench.py --graph 0 --steps 1 --warmup 1 --cpu-baseline 0 --no-roofline`):
  FETCH_DIR: --pmc FETCH_SIZE     WRITE_DIR: --pmc WRITE_SIZE
  MFMA_DIR:  --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE (optional)
Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE is in KiB and on gfx950 reports
half the bytes of a wide coalesced streaming read -> bytes = 2 * 1024 * FETCH_SIZE;
WRITE_SIZE is in KiB and exact for 16-B-per-lane stores -> bytes = 1024 * WRITE_SIZE.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def family(name):
    if "gemm_kernel" in name:
        return "gemm_kernel"
    n = name.split("(")[0]
    for tok in ("(anonymous namespace)::", "void ", "_ZN12_GLOBAL__N_1"):
        n = n.replace(tok, "")
    return n.strip()[:60]


def load(d):
    """{dispatch_id: (kernel name, {counter: value})} summed over the dispatch's rows."""
    f = sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True))
    if not f:
        raise SystemExit("no counter_collection.csv under " + d)
    out = {}
    with open(f[0]) as fh:
        for r in csv.DictReader(fh):
            did = int(r.get("Dispatch_Id") or r.get("Correlation_Id"))
            name = r["Kernel_Name"]
            c = r["Counter_Name"]
            v = float(r["Counter_Value"])
            e = out.setdefault(did, (name, defaultdict(float)))
            e[1][c] += v
    return out


def main():
    args = sys.argv[1:]
    # the profiled command runs --warmup 1 + --steps 1 eager steps = TWO steps (816 GEMM
    # launches = 2 x 408): per-step totals divide by this
    steps = 2
    if "--steps" in args:
        i = args.index("--steps")
        steps = int(args[i + 1])
        del args[i:i + 2]
    fetch = load(args[0])
    write = load(args[1])
    mfma = load(args[2]) if len(args) > 2 else {}
    fam = defaultdict(lambda: defaultdict(float))
    for did, (name, cs) in fetch.items():
        f = fam[family(name)]
        f["launches"] += 1
        f["read_bytes"] += 2.0 * 1024.0 * cs.get("FETCH_SIZE", 0.0)
    for did, (name, cs) in write.items():
        fam[family(name)]["write_bytes"] += 1024.0 * cs.get("WRITE_SIZE", 0.0)
    for did, (name, cs) in mfma.items():
        f = fam[family(name)]
        for k, v in cs.items():
            f[k] += v
    res = {}
    for k, f in fam.items():
        n = max(f["launches"], 1)
        e = {"launches": int(f["launches"]),
             "read_bytes_per_launch": f["read_bytes"] / n,
             "write_bytes_per_launch": f["write_bytes"] / n,
             "traffic_bytes_per_launch": (f["read_bytes"] + f["write_bytes"]) / n,
             "traffic_bytes_total": f["read_bytes"] + f["write_bytes"]}
        if "SQ_VALU_MFMA_BUSY_CYCLES" in f and f.get("GRBM_GUI_ACTIVE"):
            # MFMA_BUSY = matrix-pipe cycles summed over every SIMD (32 per 32x32x16 bf16 MFMA);
            # GRBM_GUI_ACTIVE is summed over the 8 XCDs -> /8 = elapsed GPU cycles.
            # utilisation = busy / (1024 SIMDs * elapsed cycles)
            e["mfma_util"] = f["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024.0 * f["GRBM_GUI_ACTIVE"] / 8.0)
        for c in ("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CU_CYCLES", "GRBM_GUI_ACTIVE"):
            if c in f:
                e[c] = f[c]
        res[k] = e
    tot = sum(e["traffic_bytes_total"] for e in res.values())
    out = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over %d eager train steps "
                     "(bench.py --graph 0 --steps 1 --warmup 1: one warm-up + one timed step), gfx950 "
                     "FETCH_SIZE x2 correction" % steps,
           "profiled_steps": steps,
           "profiled_traffic_bytes": tot,
           "step_traffic_bytes": tot / steps,
           "families": dict(sorted(res.items(), key=lambda kv: -kv[1]["traffic_bytes_total"]))}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
