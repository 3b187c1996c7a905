#!/bin/bash
# Tile-config sweep of the step's forward / dgrad conv shapes (tools/gemm_probe.py).
for s in aspp_fwd asppb_fwd l4_fwd l4_1x1_fwd l4b_1x1_fwd l3_fwd l3_1x1_fwd l3b_1x1_fwd l2_fwd l2_1x1_fwd l2b_1x1_fwd l1_fwd l1_1x1_fwd l1b_1x1_fwd aspp_dgrad l4_dgrad l3d_dgrad l3d_1x1_dgrad l3bd_1x1_dgrad; do
  line="$s"
  for c in -1 1 2 3 4 5 8 9 10 11 12 13 14 15; do
    r=$(timeout -k 5 60 python3 tools/gemm_probe.py $s $c 30 2>/dev/null | awk '{print $6}')
    line="$line $c:$r"
  done
  echo "$line"
done
