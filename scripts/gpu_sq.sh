#!/bin/bash
# SQ stall / MFMA-busy / LDS-conflict counters of one priced launch (kernels_for_pmc.py LEG S)
# Usage: gpurun -- bash scripts/gpu_sq.sh TAG LEG [S]
set -o pipefail
TAG=$1; LEG=$2; S=${3:-128}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
P="rocprofv3 -f csv --kernel-trace"
timeout -k 10 300 $P --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d $OUT/sq1_$LEG -o run -- python3 scripts/kernels_for_pmc.py $LEG $S > $OUT/sq1_$LEG.log 2>&1 || { tail -20 $OUT/sq1_$LEG.log; exit 1; }
timeout -k 10 300 $P --pmc SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT -d $OUT/sq2_$LEG -o run -- python3 scripts/kernels_for_pmc.py $LEG $S > $OUT/sq2_$LEG.log 2>&1 || { tail -20 $OUT/sq2_$LEG.log; exit 1; }
timeout -k 10 300 $P --pmc SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA -d $OUT/sq3_$LEG -o run -- python3 scripts/kernels_for_pmc.py $LEG $S > $OUT/sq3_$LEG.log 2>&1 || { tail -20 $OUT/sq3_$LEG.log; echo "sq3 failed (optional)"; }
python3 - "$OUT" "$LEG" <<'PY'
import csv, glob, sys
out, leg = sys.argv[1], sys.argv[2]
for f in sorted(glob.glob(f"{out}/sq*_{leg}/run_counter_collection.csv")):
    rows = list(csv.DictReader(open(f)))
    names = sorted({r["Kernel_Name"] for r in rows})
    for kn in names:
        if "conv_gemm" not in kn and "line_fwd" not in kn and "wgrad" not in kn:
            continue
        ds = sorted({int(r["Dispatch_Id"]) for r in rows if r["Kernel_Name"] == kn})[-3:]
        agg = {}
        for r in rows:
            if r["Kernel_Name"] == kn and int(r["Dispatch_Id"]) in ds:
                agg[r["Counter_Name"]] = agg.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"]) / len(ds)
        print(kn[:70], {k: f"{v:.4g}" for k, v in sorted(agg.items())})
PY
