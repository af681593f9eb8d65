#!/bin/bash
# same-box step A/B of weight-gradient tuning builds (128^3 graph step, 64^3
# step, 256^3 slab step): libm3d.so vs libm3d_minm128.so vs libm3d_sk16.so
set -o pipefail
OUT=gpurun_out/${1:-r06sweep}
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # lib size
  timeout -k 10 240 env M3D_LIB_FILE=$1 python -u bench.py --steps 20 --warmup 3 --size $2 --no-extras --slab-size 0 > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; return 1; }
  python3 -c "
import json; d = json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('$1 $2 step', d['ms_per_step'], 'ms (graph)', 'eager', d.get('eager_ms_per_step'))" | tee -a $OUT/summary.txt
}
for rep in 1 2; do for lib in libm3d.so libm3d_minm128.so libm3d_sk16.so; do step $lib 128 || exit 1; step $lib 64 || exit 1; done; done
for lib in libm3d.so libm3d_minm128.so libm3d_sk16.so; do
  M3D_LIB_FILE=$lib timeout -k 10 400 python -u scripts/r06/mod_ab.py - > $OUT/s.txt 2> $OUT/slab.err || { tail -20 $OUT/slab.err; exit 1; }
  echo "$lib 256 $(cat $OUT/s.txt | tr '\n' ' ')" | tee -a $OUT/summary.txt
done
