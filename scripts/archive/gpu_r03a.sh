#!/bin/bash
# Round-3 new parity tests (configs[0], configs[3], 128^3 gradients, targets, determinism) on the GPU.
set -o pipefail
OUT=gpurun_out/${1:-r03a}
mkdir -p $OUT
export TMPDIR=/tmp
PT="python -u -m pytest -x -v -s --timeout 900 --timeout-method thread"
timeout -k 10 600 $PT tests/test_gpu_config0.py tests/test_gpu_roi_nms.py tests/test_gpu_targets.py tests/test_gpu_determinism.py > $OUT/pytest_a.log 2>&1 || { echo "stage a failed"; tail -60 $OUT/pytest_a.log; exit 1; }
tail -3 $OUT/pytest_a.log
timeout -k 10 900 $PT tests/test_gpu_config3.py > $OUT/pytest_b.log 2>&1 || { echo "stage b failed"; tail -60 $OUT/pytest_b.log; exit 1; }
tail -3 $OUT/pytest_b.log
timeout -k 10 900 $PT tests/test_gpu_configs.py tests/test_gpu_conv.py > $OUT/pytest_c.log 2>&1 || { echo "stage c failed"; tail -60 $OUT/pytest_c.log; exit 1; }
tail -3 $OUT/pytest_c.log
echo DONE
