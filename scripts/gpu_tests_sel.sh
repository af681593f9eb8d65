#!/bin/bash
# Selected GPU test files (and optional -k EXPR), no bench.
# Usage: gpurun -- bash scripts/gpu_tests_sel.sh TAG "tests/a.py tests/b.py" [EXPR]
set -o pipefail
TAG=$1; FILES=$2; EXPR=${3:-}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
K=()
[ -n "$EXPR" ] && K=(-k "$EXPR")
timeout -k 10 1000 python -u -m pytest -x -v -s --timeout 900 --timeout-method thread -m gpu $FILES "${K[@]}" > $OUT/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|rel err|gradients:|kept of|forward [0-9.]+ s|vs 256|passed|failed" $OUT/pytest.log | tail -60
exit $rc
