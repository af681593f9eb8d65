#!/bin/bash
# Where the batched bias reductions' flushes land vs the graph replay's slowdown
# (nn.BIAS_BATCHED, nn.BIAS_BATCH_MAX), same box.
set -o pipefail
OUT=gpurun_out/${1:-r05bias2}
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
for sw in nn.BIAS_BATCHED=0 nn.BIAS_BATCHED=1 nn.BIAS_BATCHED=1,nn.BIAS_BATCH_MAX=4 nn.BIAS_BATCHED=1,nn.BIAS_BATCH_MAX=2; do
  timeout -k 10 240 python -u scripts/bench_ab.py $sw -- --steps 20 --warmup 3 --no-extras --slab-size 0 > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  python3 -c "
import json; d = json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('$sw', d['ms_per_step'], 'ms (graph)', 'eager', d.get('eager_ms_per_step'))" | tee -a $OUT/summary.txt
done
done
