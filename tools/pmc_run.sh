#!/bin/bash
# PMC passes (one counter group per run, separate processes) over one eager bench step.
# Usage (on the GPU box, from the repo root): bash tools/pmc_run.sh OUTDIR
set -e
OUT=${1:-gpurun_out/pmc}
mkdir -p $OUT
export TMPDIR=/tmp
CMD="python3 bench.py --graph 0 --steps 1 --warmup 1 --cpu-baseline 0 --no-roofline"
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $CMD > $OUT/fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $CMD > $OUT/write.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/mfma -o run -- $CMD > $OUT/mfma.log 2>&1
python3 tools/pmc_summary.py --steps 2 $OUT/fetch $OUT/write $OUT/mfma > $OUT/summary.json
