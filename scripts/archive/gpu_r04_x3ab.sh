#!/bin/bash
# x3 GEMM A/B: python scripts/x3_ab.py over the given make-ab libraries.
# Usage: gpurun -- bash scripts/archive/gpu_r04_x3ab.sh TAG lib1.so lib2.so ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/x3_ab.py "$@" > $OUT/x3ab.log 2>&1 || { tail -20 $OUT/x3ab.log; exit 1; }
grep -v amdgpu.ids $OUT/x3ab.log | head -20
