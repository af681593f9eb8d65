#!/bin/bash
# PyramidROIAlign 7^3 in wave-sorted order (libm3d_s3.so, M3D_TUNE_ROI_SORT=3) vs the
# default launch order: time (roi_ab.py) and PMC HBM traffic at 256^3 (separate passes).
set -o pipefail
OUT=gpurun_out/${1:-r04_roi7}
mkdir -p $OUT
export TMPDIR=/tmp
for lib in libm3d.so libm3d_s3.so libm3d.so libm3d_s3.so; do
  M3D_LIB_FILE=$lib timeout -k 10 300 python -u scripts/roi_ab.py > $OUT/one.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
  echo "$lib $(cat $OUT/one.json)"
done
for lib in libm3d.so libm3d_s3.so; do
  export M3D_LIB_FILE=$lib
  timeout -k 10 300 rocprofv3 -f csv --pmc FETCH_SIZE --kernel-trace -d $OUT/f_$lib -o run -- python3 scripts/kernels_for_pmc.py roi7 256 > $OUT/f_$lib.log 2>&1 || { tail -20 $OUT/f_$lib.log; exit 1; }
  timeout -k 10 300 rocprofv3 -f csv --pmc WRITE_SIZE --kernel-trace -d $OUT/w_$lib -o run -- python3 scripts/kernels_for_pmc.py roi7 256 > $OUT/w_$lib.log 2>&1 || { tail -20 $OUT/w_$lib.log; exit 1; }
  python3 scripts/pmc_traffic.py $OUT/f_$lib/run_counter_collection.csv $OUT/w_$lib/run_counter_collection.csv line_fwd_sl_kernel roi7_$lib $OUT/traffic.json 3 || exit 1
  rm -f $OUT/?_$lib/run_kernel_trace.csv
done
unset M3D_LIB_FILE
cat $OUT/traffic.json
