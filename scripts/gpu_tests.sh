#!/bin/bash
# GPU parity tests in stages (new / slab / all), each under its own time limit,
# logs under gpurun_out/TAG.  Usage: gpurun -- bash scripts/gpu_tests.sh TAG [stages]
set -o pipefail
TAG=${1:-r02}
STAGES=${2:-"new slab all"}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
PT="python -u -m pytest -x -v -s --timeout 1100 --timeout-method thread"
for st in $STAGES; do
  case $st in
    new)  ARGS="tests/test_gpu_optim.py tests/test_gpu_configs.py"; LIM=900;;
    slab) ARGS="tests/test_gpu_slab.py"; LIM=1200;;
    all)  ARGS="tests -m gpu"; LIM=1200;;
    *)    ARGS="$st"; LIM=900;;
  esac
  LOG=$OUT/pytest_$(echo $st | tr "/." "__").log
  echo "== $st"
  timeout -k 10 $LIM $PT $ARGS > $LOG 2>&1 || { echo "stage $st failed"; tail -80 $LOG; exit 1; }
  tail -3 $LOG
done
echo DONE
