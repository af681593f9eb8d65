#!/bin/bash
# Slab halo-plane kernels (unit tests, then the sharded-RPN tests) and the
# ROIAlign forward variants.
set -o pipefail
OUT=gpurun_out/r03h
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_slab_halo.py -m gpu > $OUT/halo.log 2>&1 || { tail -40 $OUT/halo.log; exit 1; }
tail -3 $OUT/halo.log
bash scripts/gpu_roi_sort.sh r03h/roi "M3D_ROI_SORT=0 M3D_ROI_STAGE=0" "M3D_ROI_SORT=0 M3D_ROI_STAGE=1" "M3D_ROI_SORT=3 M3D_ROI_STAGE=0" "M3D_ROI_SORT=3 M3D_ROI_STAGE=1" || exit 1
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 800 --timeout-method thread tests/test_gpu_slab.py -m gpu > $OUT/slab.log 2>&1 || { tail -40 $OUT/slab.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" $OUT/slab.log | tail -6
