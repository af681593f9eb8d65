#!/bin/bash
# GPU parity tests + the default bench line.  Usage: gpurun -- bash scripts/gpu_test_bench.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
K=${2:+-k "$2"}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread $K > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
M3D_STEP_ROOFLINE_TABLE=$OUT/step_roofline_128.json M3D_STEP_ROOFLINE_TABLE_256=$OUT/step_roofline_256.json timeout -k 10 500 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
