#!/bin/bash
# PMC of the PyramidROIAlign 14^3 launch at 256^3 (512 ROIs) per M3D_ROI_SORT order:
# FETCH_SIZE, WRITE_SIZE and the L2 hit / miss counts, each pass on its own.
set -o pipefail
OUT=gpurun_out/${1:-roipmc}
mkdir -p $OUT
export TMPDIR=/tmp
for v in 0 3; do
  for c in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
    tag=$(echo $c | cut -d' ' -f1)
    M3D_ROI_SORT=$v timeout -s KILL 120 rocprofv3 -f csv --pmc $c --kernel-trace -d $OUT/p${v}_$tag -o run -- python3 scripts/kernels_for_pmc.py roi14 256 > $OUT/p${v}_$tag.log 2>&1 || { echo "pmc $v $c failed"; tail -20 $OUT/p${v}_$tag.log; exit 1; }
    python3 - $OUT/p${v}_$tag/run_counter_collection.csv "$v $c" <<'PY'
import csv, sys, collections
vals = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    if "line_fwd" in r["Kernel_Name"]:
        vals[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
last = [vals[d] for d in sorted(vals)][-3:]
agg = {k: sum(v[k] for v in last) / len(last) for k in last[0]}
print(sys.argv[2], {k: round(v) for k, v in agg.items()})
PY
  done
done
