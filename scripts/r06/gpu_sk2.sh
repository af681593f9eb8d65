#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-r06sk2}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py -m gpu -x -q -k "wgrad or stream_k" --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -n 1 $OUT/pytest.log
leg() {
  timeout -k 10 120 python -u scripts/kernels_for_pmc.py $1 128 > $OUT/k.json 2> $OUT/k.err || { tail -20 $OUT/k.err; return 1; }
  python3 -c "
import ast; d = ast.literal_eval(open('$OUT/k.json').read().strip().splitlines()[-1]); print('$1', d['avg_launch_ms'], 'ms', d['achieved'], 'TF/s', d['frac'])" | tee -a $OUT/summary.txt
}
leg wgrad || exit 1
timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-extras --slab-size 0 > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
python3 -c "
import json; d = json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('step', d['ms_per_step'], 'ms (graph)', 'eager', d.get('eager_ms_per_step'))" | tee -a $OUT/summary.txt
timeout -k 10 300 python -u scripts/r06/legs.py > $OUT/legs.txt 2> $OUT/legs.err || { tail -30 $OUT/legs.err; exit 1; }
cat $OUT/legs.txt | cut -c1-300
timeout -k 10 600 python -u -m pytest tests/test_gpu_determinism.py tests/test_gpu_configs.py -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > $OUT/pytest2.log 2>&1 || { tail -30 $OUT/pytest2.log; exit 1; }
tail -n 1 $OUT/pytest2.log
