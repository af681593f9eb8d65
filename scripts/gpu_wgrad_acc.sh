#!/bin/bash
# Winograd weight-gradient accuracy vs float64 under both tile choices
set -o pipefail
OUT=gpurun_out/${1:-wgradacc}
mkdir -p $OUT
export TMPDIR=/tmp
for nz in 2 4; do
  M3D_WINO_WGRAD_NZ=$nz timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_gpu_conv.py -k "wino_weight_gradient_accuracy" -m gpu > $OUT/t$nz.log 2>&1 || { tail -30 $OUT/t$nz.log; exit 1; }
  echo "NZ=$nz"; grep -E "rel err|passed|failed" $OUT/t$nz.log
done
