#!/bin/bash
# bench.py measurement-order probe (tools/bench_order_probe.py), one process per order
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
for ord in fp8,fp8 c3,fp8,fp8 c3,sleep5,fp8 bf16,fp8; do
  echo "== $ord" >> $O/order.txt
  timeout -k 10 400 python tools/bench_order_probe.py $ord 8 >> $O/order.txt 2>/dev/null || exit 1
done
