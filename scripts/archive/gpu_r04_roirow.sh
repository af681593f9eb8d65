#!/bin/bash
# PyramidROIAlign forward: line kernel (libm3d.so) vs the separable row form
# (libm3d_row.so, M3D_TUNE_ROI_ROW=2); outputs must agree bit for bit (sha).
set -o pipefail
OUT=gpurun_out/${1:-r04_roirow}
mkdir -p $OUT
export TMPDIR=/tmp
LIBS=${2:-"libm3d.so libm3d_row.so"}
for lib in $LIBS $LIBS; do
  M3D_LIB_FILE=$lib timeout -k 10 300 python -u scripts/roi_ab.py > $OUT/one.json 2>> $OUT/roi_ab.err || { echo "$lib failed"; tail -20 $OUT/roi_ab.err; exit 1; }
  echo "$lib $(cat $OUT/one.json)" | tee -a $OUT/roi_ab.jsonl
done
M3D_LIB_FILE=${3:-libm3d_row.so} timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_roi_nms.py tests/test_gpu_config3.py -k "pyramid or roi or align" > $OUT/pytest_row.log 2>&1; rc=$?
tail -3 $OUT/pytest_row.log
exit $rc
