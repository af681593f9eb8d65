#!/bin/bash
# Step-time A/B: eager launches vs the HIP-graph replayed step (bench --graph), 128^3, twice.
set -o pipefail
OUT=gpurun_out/${1:-r04_graph}
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
for g in "" "--graph"; do
  timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-extras --slab-size 0 $g > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  python3 -c "
import json; d = json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('graph=[$g]', 'step', d['ms_per_step'], 'ms', d['value'], 'vol/s')"
done
done
