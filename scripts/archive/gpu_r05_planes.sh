#!/bin/bash
# Batched split planes (nn.X3Planes): GPU tests, the model / gradient tests, a
# same-box step A/B (graph + eager).
set -o pipefail
OUT=gpurun_out/${1:-r05planes}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py -k "x3_planes or col_sums or bias_batch" -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -n 1 $OUT/pytest.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_model.py tests/test_gpu_determinism.py tests/test_gpu_bnfuse.py tests/test_gpu_slab.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest2.log 2>&1 || { tail -40 $OUT/pytest2.log; exit 1; }
tail -n 1 $OUT/pytest2.log
for rep in 1 2; do
for sw in nn.X3_PLANES_BATCHED=1 nn.X3_PLANES_BATCHED=0; do
  timeout -k 10 240 python -u scripts/bench_ab.py $sw -- --steps 20 --warmup 3 --no-extras --slab-size 0 > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  python3 -c "
import json; d = json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('$sw', d['ms_per_step'], 'ms (graph)', 'eager', d.get('eager_ms_per_step'))" | tee -a $OUT/summary.txt
done
done
