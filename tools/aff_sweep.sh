for c in -1 0 1 2 3 4 5 8 9 10 11 12 13 14 15; do timeout -k 5 60 python3 tools/gemm_probe.py affinity $c 50 2>/dev/null; done
