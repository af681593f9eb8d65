#!/bin/bash
# Per-layer conv table (scripts/conv_layers.py) at SIZE for each library build.
# Usage: gpurun -- bash scripts/archive/gpu_r05_layers.sh TAG SIZE libm3d.so libm3d_X.so ...
set -o pipefail
TAG=$1; SIZE=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for L in "$@"; do
  M3D_LIB_FILE=$L timeout -k 10 400 python -u scripts/conv_layers.py --size $SIZE --reps 3 > $OUT/layers${SIZE}_$L.txt 2>&1 || { tail -20 $OUT/layers${SIZE}_$L.txt; exit 1; }
  echo "$L $(tail -1 $OUT/layers${SIZE}_$L.txt)"
done
