#!/bin/bash
# Tile-pair interleave in the 128x128 x3 GEMMs (libm3d_pt.so: M3D_TUNE_X3_PAIR_TILES=1)
# vs the default build: parity tests on the quad build, then the priced launch and
# the step, same box.
set -o pipefail
OUT=gpurun_out/${1:-r05pt}
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
for lib in libm3d.so libm3d_pt.so; do
  timeout -k 10 120 env M3D_LIB_FILE=$lib python -u scripts/kernels_for_pmc.py wgrad 128 > $OUT/k.json 2> $OUT/k.err || { tail -20 $OUT/k.err; exit 1; }
  python3 -c "
import ast; d = ast.literal_eval(open('$OUT/k.json').read().strip().splitlines()[-1]); print('$lib wgrad', d['avg_launch_ms'], 'ms', d['achieved'], 'TF/s', d['frac'])" | tee -a $OUT/summary.txt
  timeout -k 10 240 env M3D_LIB_FILE=$lib python -u bench.py --steps 20 --warmup 3 --no-extras --slab-size 0 > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  python3 -c "
import json; d = json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('$lib step', d['ms_per_step'], 'ms (graph)', 'eager', d.get('eager_ms_per_step'))" | tee -a $OUT/summary.txt
done
done
