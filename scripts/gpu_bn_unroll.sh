#!/bin/bash
# bn_act_bwd_kernel row unroll (BN_UNROLL 2 default vs the 1 / 4 A/B builds):
# BN / model gradient tests, then the 128^3 step A/B.
set -o pipefail
OUT=gpurun_out/bnu
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_conv.py tests/test_gpu_model.py tests/test_gpu_determinism.py > $OUT/pytest.log 2>&1 \
    || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
bash scripts/gpu_step_ab.sh bnu_ab "M3D_LIB_FILE=libm3d.so" "M3D_LIB_FILE=libm3d_bn1.so" "M3D_LIB_FILE=libm3d_bn4.so"
