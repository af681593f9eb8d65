#!/bin/bash
# Winograd transform kernels per variant (M3D_WINO_XCD, the NT=0 A/B build) on
# the P2 RPN conv shapes: rocprofv3 kernel stats per run.
set -o pipefail
OUT=gpurun_out/winox
mkdir -p $OUT
export TMPDIR=/tmp
for shape in 32,32,32,256,512 32,32,32,64,64; do
for v in "M3D_WINO_XCD=0" "M3D_WINO_XCD=1" "M3D_LIB_FILE=libm3d_nt0.so"; do
  tag=$(echo "$shape-$v" | tr ',=.' '___')
  env $v SHAPE=$shape timeout -k 10 120 rocprofv3 -f csv --kernel-trace --stats -d $OUT/$tag -o run -- python3 scripts/wino_xform_bench.py > $OUT/$tag.log 2>&1 || { tail -20 $OUT/$tag.log; exit 1; }
  echo "== $shape $v: $(grep shape $OUT/$tag.log)"
  python3 - "$OUT/$tag/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if "wino_input" in n or "wino_output" in n or "x3_gemm" in n:
        print(f"   {float(r['AverageNs']) / 1e3:8.1f} us x{r['Calls']:>4}  {n.split('(')[0][-50:]}")
PY
done
done
