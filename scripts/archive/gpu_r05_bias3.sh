#!/bin/bash
# Batched bias reductions with a 4-item kernel-argument table (M3D_COL_SUMS_MAX 4)
# vs per-unit, graph + eager, same box; their GPU tests first.
set -o pipefail
OUT=gpurun_out/${1:-r05bias3}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py -k "col_sums or bias_batch" -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -n 1 $OUT/pytest.log
for rep in 1 2; do
for sw in nn.BIAS_BATCHED=0 nn.BIAS_BATCHED=1; do
  timeout -k 10 240 python -u scripts/bench_ab.py $sw -- --steps 20 --warmup 3 --no-extras --slab-size 0 > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  python3 -c "
import json; d = json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('$sw', d['ms_per_step'], 'ms (graph)', 'eager', d.get('eager_ms_per_step'))" | tee -a $OUT/summary.txt
done
done
