#!/bin/bash
# Step-time and per-layer A/B of library builds (make ab AB_NAME=X AB_DEFS=...):
# GPU tests EXPR under the default library, then for each library file the
# per-layer conv table and two short bench runs.
# Usage: gpurun -- bash scripts/gpu_ab_libs.sh TAG "EXPR" libm3d.so libm3d_X.so ...
set -o pipefail
TAG=$1; EXPR=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$EXPR" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu -k "$EXPR" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
  tail -n 1 $OUT/pytest.log
fi
for L in "$@"; do
  M3D_LIB_FILE=$L timeout -k 10 200 python scripts/conv_layers.py --size 128 > $OUT/layers_$L.txt 2>&1 || { tail -20 $OUT/layers_$L.txt; exit 1; }
done
for rep in 1 2; do
for L in "$@"; do
  M3D_LIB_FILE=$L timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-extras --slab-size 0 > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  python3 -c "
import json; d = json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('$L step', d['ms_per_step'], 'ms')"
done
done
