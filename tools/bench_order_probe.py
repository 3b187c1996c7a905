"""Why a recorded configs[3] co-attention graph run before bench.py's fp8 extra line made that line
8 % slower (round 5: 152 vs 166 frame-pairs/s; bench.py then ran configs[3] last).

    python tools/bench_order_probe.py ORDER [steps]

ORDER is a comma list of legs run in one process: fp8 (bench.extra_line(dev, 8, 473, "fp8")),
c3 (bench.coattention_roofline: the 20-launch graph, released after), sleepN (N seconds idle),
bf16 (extra_line at B = 4 bf16).  Each leg prints its
rate, the allocator's reserved / allocated bytes and the allocator's retry / split counters
before and after, so pool state, fragmentation and a clock / power effect (recovers after an
idle gap) can be told apart."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch

import bench


def mem():
    s = torch.cuda.memory_stats()
    return "reserved %.2f GB alloc %.2f GB retries %d inactive_split %.2f GB segments %d" % (
        torch.cuda.memory_reserved() / 1e9, torch.cuda.memory_allocated() / 1e9,
        s.get("num_alloc_retries", 0), s.get("inactive_split_bytes.all.current", 0) / 1e9,
        s.get("segment.all.current", 0))


def main():
    order = sys.argv[1].split(",")
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    dev = torch.device("cuda:0")
    keep = []
    for leg in order:
        t0 = time.perf_counter()
        before = mem()
        if leg == "fp8" or leg == "bf16":
            r = bench.extra_line(dev, 8 if leg == "fp8" else 4, 473, leg, steps=steps)
            res = "%.1f pairs/s (%.1f ms/step)" % (r["value"], r["ms_per_step"])
        elif leg.startswith("c3"):
            r = bench.coattention_roofline(dev)
            res = "configs[3] %.1f us/launch" % r["us_per_launch"]
        elif leg.startswith("sleep"):
            torch.cuda.synchronize()
            time.sleep(float(leg[5:]))
            res = "idle"
        else:
            raise SystemExit("unknown leg " + leg)
        torch.cuda.synchronize()
        print("%-8s %-36s %5.1f s | before: %s | after: %s" % (leg, res, time.perf_counter() - t0, before, mem()),
              flush=True)


if __name__ == "__main__":
    main()
