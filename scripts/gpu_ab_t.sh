#!/bin/bash
# gpu tests (-k) then A/B of an env switch: gpu_ab_t.sh TAG KEXPR VAR A B
set -o pipefail
TAG=$1; KEXPR=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q -k "$KEXPR" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
bash scripts/gpu_ab.sh $TAG "$@"
