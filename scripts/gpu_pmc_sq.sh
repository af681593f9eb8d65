#!/bin/bash
# SQ/LDS PMC passes (separate rocprofv3 runs, kernel-trace only) over one bench leg.
# Usage: gpurun -- bash scripts/gpu_pmc_sq.sh LEG S KERNEL_SUBSTR TAG
set -o pipefail
export TMPDIR=/tmp
LEG=$1; S=$2; KS=$3; TAG=${4:-sq}
O=gpurun_out/$TAG; mkdir -p $O
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_CYCLES"
P2="SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_LEVEL_WAVES SQ_INSTS_VALU"
P3="SQ_WAVES SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_LDS_ADDR_CONFLICT SQ_BUSY_CU_CYCLES"
i=0
for pass in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 -f csv --pmc $pass --kernel-trace -d $O/p$i -o run -- python3 scripts/kernels_for_pmc.py $LEG $S > $O/p$i.log 2>&1 || { tail -20 $O/p$i.log; exit 1; }
  python3 - $O/p$i/run_counter_collection.csv "$KS" <<'PY'
import csv, sys, collections
rows = [r for r in csv.DictReader(open(sys.argv[1])) if sys.argv[2] in r["Kernel_Name"]]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    agg[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
last = sorted(agg)[-1]
print(rows[-1]["Kernel_Name"][:60], {k: f"{v:.4g}" for k, v in agg[last].items()})
PY
  rm -f $O/p$i/run_kernel_trace.csv
done
