#!/bin/bash
# PMC passes (separate runs) of the PyramidROIAlign leg at S=256, pool 14, per variant.
set -o pipefail
export TMPDIR=/tmp ROI_CASES="256,512" ROI_POOLS="14" ROI_REPS=3
O=gpurun_out/roi_pmc; mkdir -p $O
for v in ${1:-0 5}; do
  for ctr in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
    tag=$(echo $ctr | tr ' ' '_')
    M3D_ROI_VARIANT=$v timeout -k 10 120 rocprofv3 -f csv --pmc $ctr --kernel-trace -d $O/v${v}_$tag -o run -- python3 scripts/roi_variants.py > $O/v${v}_$tag.log 2>&1 || { tail -20 $O/v${v}_$tag.log; exit 1; }
    python3 - $O/v${v}_$tag/run_counter_collection.csv "$v" <<'PY'
import csv, sys, collections
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "fwd_kernel" in r["Kernel_Name"]]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    agg[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
last = sorted(agg, key=int)[-1]
print("variant", sys.argv[2], rows[0]["Kernel_Name"][:40], dict(agg[last]))
PY
  done
done
