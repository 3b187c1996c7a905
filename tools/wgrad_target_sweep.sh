#!/bin/bash
# wgrad K-split target sweep (blocks) on the step's weight-gradient shapes (batch 4 frames).
for s in l1w_wgrad l1w_1x1_wgrad l1wb_1x1_wgrad l2w_1x1_wgrad l2wb_1x1_wgrad l3w_1x1_wgrad l3wb_1x1_wgrad l3w_wgrad asppw_wgrad; do
  line="$s"
  for t in 128 256 512 1024; do
    r=$(timeout -k 5 60 python3 tools/gemm_probe.py $s -1 30 $t 2>/dev/null | awk '{print $6}')
    line="$line $t:$r"
  done
  echo "$line"
done
