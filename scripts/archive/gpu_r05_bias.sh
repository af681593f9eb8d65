#!/bin/bash
# Batched bias-only reductions (nn.BiasSums / m3d_col_sums_batched): their GPU
# tests, the model/gradient tests that cover them, a same-box step A/B, and the
# 256^3 forward roofline.
set -o pipefail
OUT=gpurun_out/${1:-r05bias}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py -k "col_sums or bias_batch or bn_affine_batched" -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -n 1 $OUT/pytest.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_model.py tests/test_gpu_determinism.py tests/test_gpu_dp.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest2.log 2>&1 || { tail -40 $OUT/pytest2.log; exit 1; }
tail -n 1 $OUT/pytest2.log
for rep in 1 2; do
for sw in nn.BIAS_BATCHED=1 nn.BIAS_BATCHED=0; do
  timeout -k 10 240 python -u scripts/bench_ab.py $sw -- --steps 20 --warmup 3 --no-extras --slab-size 0 > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  python3 -c "
import json; d = json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('$sw', d['ms_per_step'], 'ms (graph)', 'eager', d.get('eager_ms_per_step'))" | tee -a $OUT/summary.txt
done
done
timeout -k 10 300 python -u scripts/fwd_roofline_256.py 256 > $OUT/fwd256.json 2> $OUT/fwd256.err || { tail -20 $OUT/fwd256.err; exit 1; }
python3 -c "
import json; d = json.loads(open('$OUT/fwd256.json').read().strip().splitlines()[-1]); print({k: (v['ms'], v['roofline_ms'], v['frac_roofline']) for k, v in d.items()})"
