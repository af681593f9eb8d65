#!/bin/bash
# same-box A/B: libm3d.so (working tree) vs libm3d_prev.so (last commit)
set -o pipefail
OUT=gpurun_out/${1:-r06abprev}
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  timeout -k 10 240 env M3D_LIB_FILE=$1 python -u bench.py --steps 20 --warmup 3 --no-extras --slab-size 0 > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; return 1; }
  python3 -c "
import json; d = json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('$1 step', d['ms_per_step'], 'ms (graph)', 'eager', d.get('eager_ms_per_step'))" | tee -a $OUT/summary.txt
}
c0() {
  timeout -k 10 200 env M3D_LIB_FILE=$1 python -u scripts/r06/c0_time.py > $OUT/c0.txt 2>&1 || { tail -20 $OUT/c0.txt; return 1; }
  echo "$1 c0 $(tail -2 $OUT/c0.txt | tr '\n' ' ')" | tee -a $OUT/summary.txt
}
for rep in 1 2; do for lib in libm3d_prev.so libm3d.so; do step $lib || exit 1; c0 $lib || exit 1; done; done
