#!/bin/bash
# Per-tensor gradient error tables (scripts/grad_table.py) of host variants and
# of the F(2x2x4) build (libm3d_ny2.so).  Usage: gpurun -- bash scripts/archive/gpu_r05_grad.sh TAG [variants]
set -o pipefail
TAG=${1:-r05grad}; VAR=${2:-base,wino_min128,wino_min256,no_wino}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u scripts/grad_table.py --out $OUT/grad_f424.json --variants $VAR > $OUT/grad_f424.log 2>&1 || { tail -30 $OUT/grad_f424.log; exit 1; }
cat $OUT/grad_f424.log | grep median
if [ -f 3d-mask-r-cnn_amd/m3d/libm3d_ny2.so ]; then
M3D_LIB_FILE=libm3d_ny2.so timeout -k 10 300 python -u scripts/grad_table.py --out $OUT/grad_f224.json --variants base > $OUT/grad_f224.log 2>&1 || { tail -30 $OUT/grad_f224.log; exit 1; }
cat $OUT/grad_f224.log | grep median
fi
