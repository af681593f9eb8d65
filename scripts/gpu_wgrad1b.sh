#!/bin/bash
# 1x1x1 weight gradients: m-split floor / kernel choice for small m, alone and in the 128^3 step.
set -o pipefail
OUT=gpurun_out/wg1b
mkdir -p $OUT
export TMPDIR=/tmp
SH="8,8,128,1024,256;8,8,128,256,1024;4,4,128,2048,512;4,4,128,512,2048;16,16,128,512,128;16,16,128,128,512"
for v in "M3D_X3W_TR_MINM=256" "M3D_X3W_TR_MINM=128" "M3D_X3W_TR_MINM=512" "M3D_X3W_TR_MIN_M=16384" "M3D_X3W_TR_MINM=256 M3D_X3W_TR_MIN_M=4096"; do
  echo "== $v"
  env $v SHAPES=$SH timeout -k 10 120 python3 scripts/wgrad1_bench.py > $OUT/w.log 2>&1 || { tail -20 $OUT/w.log; exit 1; }
  grep "M=" $OUT/w.log
done
bash scripts/gpu_step_ab.sh wg1b_ab "M3D_X3W_TR_MINM=64" "M3D_X3W_TR_MINM=256"
