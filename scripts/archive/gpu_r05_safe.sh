#!/bin/bash
# Staged check after a GPU fault: the x3 GEMM / conv / Winograd / BN-affine
# tests with serialized launches first (a fault names its kernel), then the
# 128^3 gradient error tables of the given libraries and short benches.
# Usage: gpurun -- bash scripts/archive/gpu_r05_safe.sh TAG libm3d.so [libm3d_X.so ...]
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
AMD_SERIALIZE_KERNEL=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "split3 or gemm or conv1_x3 or bn_affine or wino or maxpool or fused" tests/test_gpu_bnfuse.py > $OUT/stage1.log 2>&1 || { echo "stage1 failed"; tail -30 $OUT/stage1.log; exit 1; }
tail -n 1 $OUT/stage1.log
for L in "$@"; do
  M3D_LIB_FILE=$L timeout -k 10 240 python -u scripts/grad_table.py --out $OUT/grad_$L.json --variants base > $OUT/grad_$L.log 2>&1 || { tail -20 $OUT/grad_$L.log; exit 1; }
  echo "$L $(grep median $OUT/grad_$L.log | cut -c1-120)"
done
for rep in 1 2; do
for L in "$@"; do
  M3D_LIB_FILE=$L timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-extras --slab-size 0 > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  python3 -c "
import json; d = json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('$L step', d['ms_per_step'], 'ms')"
done
done
