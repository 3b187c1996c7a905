"""Co-attention kernel time from a rocprofv3 --kernel-trace CSV of the bench command: the
cross-check of bench.py's roofline_coattention_train / roofline_coattention (HIP events).

    python tools/coatt_trace_summary.py <run_kernel_trace.csv> [out.json]

Training launches (flash forward, dVa_t, PV, their split merges) are counted per step, with
the step count taken from the dVa_t<both terms> launches (one per step: the RGB encoder).
bench.py's configs[3] measurement runs after the last training step, so every co-attention
launch that starts after the last dVa_t launch belongs to it.
"""
import csv
import json
import sys

TRAIN = ("coatt_fused_fwd_k", "coatt_q48_k", "coatt_flash_dvat_k", "dvat_sum_k", "coatt_merge_k")
# the forward / PV kernel (variant 5 since round 5, variant 1 before) and its split merge
FWD0 = ("coatt_fused_fwd_k<0>", "coatt_merge_k<0>", "coatt_q48_k<0>")
PV = ("coatt_fused_fwd_k<1>", "coatt_merge_k<1>", "coatt_q48_k<1>", "dvat_sum_k")
MAIN0 = ("coatt_fused_fwd_k<0>", "coatt_q48_k<0>")
TIMED = 200   # bench.py coattention_roofline: 5 x (graph replay of 20 + 20 eager launches)


def summarise(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    name = lambda r: r["Kernel_Name"]
    dvat = [r for r in rows if "coatt_flash_dvat_k<true, true>" in name(r)]
    if not dvat:
        raise SystemExit("no dVa_t launches in " + path)
    t_last = int(dvat[-1]["Start_Timestamp"])
    steps = len(dvat)
    train = [r for r in rows if any(k in name(r) for k in TRAIN) and int(r["Start_Timestamp"]) <= t_last + 1]
    # the PV launch and its merge follow the last dVa_t of the step
    tail = [r for r in rows if int(r["Start_Timestamp"]) > t_last and
            any(k in name(r) for k in PV)]
    train += tail
    c3 = [r for r in rows if int(r["Start_Timestamp"]) > t_last and
          any(k in name(r) for k in FWD0)]
    fam = {}
    for r in train:
        k = name(r).replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        f = fam.setdefault(k, [0, 0.0])
        f[0] += 1
        f[1] += dur(r)
    c3_main = [r for r in c3 if any(k in name(r) for k in MAIN0)]
    return {"source": path, "steps": steps,
            "train_us_per_step": sum(dur(r) for r in train) / steps,
            "train_families": {k: {"launches_per_step": v[0] / steps, "us_per_step": v[1] / steps}
                               for k, v in sorted(fam.items())},
            "configs3_launches": len(c3_main),
            "configs3_us_per_launch": (sum(dur(r) for r in c3) / len(c3_main)) if c3_main else None,
            # the timed part of bench.py's configs[3] line (round 6: settling replays first, then 5
            # x (graph of 20 + 20 eager launches)): its last TIMED launches
            "configs3_timed_launches": min(len(c3_main), TIMED),
            "configs3_us_per_launch_timed": (sum(dur(r) for r in c3_main[-TIMED:]) /
                                             min(len(c3_main), TIMED)) if c3_main else None}


if __name__ == "__main__":
    s = summarise(sys.argv[1])
    print(json.dumps(s, indent=1))
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            json.dump(s, f, indent=1)
