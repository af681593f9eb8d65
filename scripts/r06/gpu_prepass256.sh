#!/bin/bash
# the 256^3 depth-slab step with / without the Winograd weight pre-pass, each
# spec in its own process (twice, alternated), and the configs[0] leg.
set -o pipefail
OUT=gpurun_out/${1:-r06pre256}
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for spec in nn.WINO_V_PREPASS=0 -; do
    timeout -k 10 400 python -u scripts/r06/mod_ab.py $spec > $OUT/s.txt 2> $OUT/slab.err || { tail -20 $OUT/slab.err; exit 1; }
    echo "$spec $(cat $OUT/s.txt | tr '\n' ' ')" | tee -a $OUT/summary.txt
  done
done
for spec in nn.WINO_V_PREPASS=0 nn.WINO_V_PREPASS=1; do
  timeout -k 10 300 python -u scripts/bench_ab.py $spec -- --steps 10 --warmup 3 --size 64 --no-extras --slab-size 0 > $OUT/c.json 2> $OUT/c.err || { tail -20 $OUT/c.err; exit 1; }
  python3 -c "
import json; d = json.loads(open('$OUT/c.json').read().strip().splitlines()[-1]); print('$spec 64^3 step', d['ms_per_step'], 'eager', d.get('eager_ms_per_step'))" | tee -a $OUT/summary.txt
done
