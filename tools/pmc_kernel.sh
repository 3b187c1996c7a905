#!/bin/bash
# PMC passes over any command, summed per launch of the kernels whose name contains FILTER.
# Usage (GPU box, repo root): bash tools/pmc_kernel.sh OUT FILTER -- cmd args...
OUT=$1; FILTER=$2; shift 3
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for P in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE" \
         "FETCH_SIZE TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum" \
         "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum" \
         "SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o run -- "$@" > $OUT/p$i.log 2>&1 || echo "pass $i failed" >> $OUT/fail.txt
done
python3 - $OUT "$FILTER" <<'PY'
import csv, glob, sys, collections
out, filt = sys.argv[1], sys.argv[2]
tot = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if filt not in r["Kernel_Name"]:
            continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
for k in sorted(tot):
    print("%-36s %16.4g  (per launch %.4g)" % (k, tot[k], tot[k] / max(n[k], 1)))
PY
