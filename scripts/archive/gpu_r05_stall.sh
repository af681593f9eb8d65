#!/bin/bash
# Where x3_wgrad_tr_kernel / x3_gemm256_af_kernel waves spend their cycles
# (MI355X_MICROARCH.md SQ table: WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES)
# and their LDS bank conflicts; one pass of <= 8 SQ counters each.
set -o pipefail
OUT=gpurun_out/${1:-r05stall}
mkdir -p $OUT
export TMPDIR=/tmp
for leg in wgrad gemm; do
  timeout -s KILL 120 rocprofv3 -f csv --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace -d $OUT/s_$leg -o run -- python3 scripts/kernels_for_pmc.py $leg 128 > $OUT/s_$leg.log 2>&1 || { tail -20 $OUT/s_$leg.log; exit 1; }
  rm -f $OUT/s_$leg/run_kernel_trace.csv
done
python3 - <<'PY'
import csv, glob, collections
for leg, kern in (("wgrad", "x3_wgrad_tr_kernel"), ("gemm", "x3_gemm256_af_kernel")):
    f = glob.glob(f"gpurun_out/r05stall/s_{leg}/**/*counter_collection.csv", recursive=True)[0]
    by = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if kern in r.get("Kernel_Name", ""):
            by[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    d = sorted(by, key=int)[-1]
    c = by[d]
    w = c["SQ_WAVE_CYCLES"]
    print(leg, kern, {k: round(v / w, 3) for k, v in c.items() if k.startswith("SQ_WAIT") or k == "SQ_ACTIVE_INST_ANY"},
          "lds conflict / lds active", round(c["SQ_LDS_BANK_CONFLICT"] / max(c["SQ_LDS_IDX_ACTIVE"], 1), 3),
          {k: c[k] for k in sorted(c)})
PY
