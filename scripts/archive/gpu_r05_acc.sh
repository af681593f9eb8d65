#!/bin/bash
# Accuracy / step-time A/B of x3 accumulation and data-gradient tile builds:
# the conv / Winograd / GEMM GPU tests under the default library, then per
# library the 128^3 gradient error table (grad_table.py) and two interleaved
# short bench runs (GRAD_LIBS / BENCH_LIBS: subsets), then the conv / Winograd / GEMM GPU tests (default library).  Usage: gpurun -- bash scripts/archive/gpu_r05_acc.sh TAG libm3d.so libm3d_X.so ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
GL=${GRAD_LIBS:-$*}
for L in $GL; do
  M3D_LIB_FILE=$L timeout -k 10 240 python -u scripts/grad_table.py --out $OUT/grad_$L.json --variants base > $OUT/grad_$L.log 2>&1 || { tail -20 $OUT/grad_$L.log; exit 1; }
  echo "$L $(grep median $OUT/grad_$L.log | cut -c1-120)"
done
BL=${BENCH_LIBS:-$*}
for rep in 1 2; do
for L in $BL; do
  M3D_LIB_FILE=$L timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-extras --slab-size 0 > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  python3 -c "
import json; d = json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('$L step', d['ms_per_step'], 'ms')"
done
done
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu -k "conv or wino or gemm or x3 or slab or grad" -p no:cacheprovider -s > $OUT/pytest.log 2>&1
grep -E "gradients:|passed|failed" $OUT/pytest.log | cut -c1-200
