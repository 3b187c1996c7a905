for s in l3_wgrad aspp_wgrad l4_wgrad l1_wgrad l2_wgrad l3_1x1_wgrad l3b_1x1_wgrad; do
  for c in -1 0 1 6 7 11 12 13 14 15 16; do
    timeout -k 5 60 python3 tools/gemm_probe.py $s $c 50 2>/dev/null || echo "$s $c FAILED"
  done
done
