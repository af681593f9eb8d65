#!/bin/bash
# full-size gradient parity (configs[0] / configs[1], with the per-tensor table
# lines) + the determinism and fused-BN model tests.  bash scripts/r06/gpu_parity.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-r06par}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_config0.py tests/test_gpu_determinism.py tests/test_gpu_bnfuse.py > $OUT/parity.log 2>&1
rc=$?
grep "gradients:" $OUT/parity.log | cut -c1-400
grep -c PASSED $OUT/parity.log
tail -3 $OUT/parity.log
exit $rc
