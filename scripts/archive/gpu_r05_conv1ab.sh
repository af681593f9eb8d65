#!/bin/bash
# Step A/B of the 1x1x1 bf16-split GEMM selection (nn.CONV1_X3_*): round-5
# thresholds vs round 4's (K >= 256, 256 tiles both ways), graph and eager,
# then the 256^3 forward roofline with each.
set -o pipefail
OUT=gpurun_out/${1:-r05conv1ab}
mkdir -p $OUT
export TMPDIR=/tmp
OLD="nn.CONV1_X3_MIN_K=256,nn.CONV1_X3_FWD_TILES=256"
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -n 1 $OUT/pytest.log
for rep in 1 2; do
for sw in nn.CONV1_X3_MIN_K=32 $OLD; do
  timeout -k 10 240 python -u scripts/bench_ab.py $sw -- --steps 20 --warmup 3 --no-extras --slab-size 0 > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  python3 -c "
import json; d = json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('$sw', d['ms_per_step'], 'ms (graph)', 'eager', d.get('eager_ms_per_step'))" | tee -a $OUT/summary.txt
done
done
for sw in nn.CONV1_X3_MIN_K=32 $OLD; do
  timeout -k 10 300 python -u scripts/fwd_roofline_256.py 256 $sw > $OUT/fwd.json 2> $OUT/fwd.err || { tail -20 $OUT/fwd.err; exit 1; }
  python3 -c "
import json; d = json.loads(open('$OUT/fwd.json').read().strip().splitlines()[-1]); print('$sw', {k: (v['ms'], v['roofline_ms'], v['frac_roofline']) for k, v in d.items()})" | tee -a $OUT/summary.txt
done
