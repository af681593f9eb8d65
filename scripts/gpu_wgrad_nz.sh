#!/bin/bash
# Weight gradient on F(2x2x4) tiles reusing the forward's kept U (M3D_WINO_WGRAD_NZ=4):
# conv / gradient-parity / determinism tests under it, then the step A/B.
set -o pipefail
OUT=gpurun_out/${1:-wgradnz}
mkdir -p $OUT
export TMPDIR=/tmp
M3D_WINO_WGRAD_NZ=4 timeout -k 10 900 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_model.py tests/test_gpu_config0.py tests/test_gpu_determinism.py "tests/test_gpu_configs.py::test_config1_gradients_full_size" -m gpu > $OUT/tests.log 2>&1 || { tail -60 $OUT/tests.log; exit 1; }
grep -E "passed|failed|worst|median|configs\[" $OUT/tests.log | tail -12
bash scripts/gpu_step_ab.sh ${1:-wgradnz}/ab "M3D_WINO_WGRAD_NZ=2" "M3D_WINO_WGRAD_NZ=4"
