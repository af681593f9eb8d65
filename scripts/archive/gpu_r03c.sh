#!/bin/bash
# ROI kernels (deterministic grad_image, region-major pyramid forward) + full-size configs tests.
set -o pipefail
OUT=gpurun_out/${1:-r03c}
mkdir -p $OUT
export TMPDIR=/tmp
PT="python -u -m pytest -x -v -s --timeout 900 --timeout-method thread"
timeout -k 10 600 $PT tests/test_gpu_roi_nms.py tests/test_gpu_heads.py > $OUT/pytest_roi.log 2>&1 || { echo "stage roi failed"; tail -60 $OUT/pytest_roi.log; exit 1; }
tail -3 $OUT/pytest_roi.log
timeout -k 10 900 $PT tests/test_gpu_configs.py > $OUT/pytest_cfg.log 2>&1 || { echo "stage cfg failed"; tail -60 $OUT/pytest_cfg.log; exit 1; }
tail -3 $OUT/pytest_cfg.log
timeout -k 10 900 $PT tests/test_gpu_config3.py > $OUT/pytest_cfg3.log 2>&1 || { echo "stage cfg3 failed"; tail -60 $OUT/pytest_cfg3.log; exit 1; }
tail -3 $OUT/pytest_cfg3.log
echo DONE
