#!/bin/bash
# F(4,3) on y (libm3d_ny4.so, M3D_TUNE_WINO_NY=4): step A/B against the default,
# then the Winograd / model parity tests on it.
set -o pipefail
OUT=gpurun_out/${1:-r04_ny4}
mkdir -p $OUT
export TMPDIR=/tmp
bash scripts/gpu_step_ab.sh ${1:-r04_ny4}_ab "M3D_LIB_FILE=libm3d.so" "M3D_LIB_FILE=libm3d_ny4.so" || exit 1
M3D_LIB_FILE=libm3d_ny4.so timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_conv.py tests/test_gpu_model.py tests/test_gpu_bnfuse.py tests/test_gpu_slab_halo.py tests/test_gpu_configs.py \
  > $OUT/pytest.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed|gradients:|rel err" $OUT/pytest.log | tail -25
exit $rc
