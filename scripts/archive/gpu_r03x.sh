#!/bin/bash
# Weight-gradient stream fork events (m3d_stream_fork): GPU tests on the
# default, then the 128^3 step A/B of the event kinds.
set -o pipefail
OUT=gpurun_out/r03x
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_gpu_model.py tests/test_gpu_dp.py tests/test_gpu_slab.py tests/test_gpu_determinism.py > $OUT/pytest.log 2>&1 \
    || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
bash scripts/gpu_step_ab.sh r03x_ab "M3D_FORK_EVENT=1" "M3D_FORK_EVENT=torch" "M3D_FORK_EVENT=2" "M3D_FORK_EVENT=0"
