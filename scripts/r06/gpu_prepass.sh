#!/bin/bash
# Winograd weight pre-pass (nn.WinoVPrep): bitwise tests, the parity subset,
# then same-box A/Bs (nn.WINO_V_PREPASS 0 / 1) at 128^3 and 256^3.
set -o pipefail
OUT=gpurun_out/${1:-r06pre}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_wino_prepass.py tests/test_gpu_determinism.py tests/test_gpu_bnfuse.py tests/test_gpu_configs.py -s > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
grep -c PASSED $OUT/tests.log; grep "gradients:" $OUT/tests.log | cut -c1-160
step() {
  timeout -k 10 240 python -u scripts/bench_ab.py $1 -- --steps 20 --warmup 3 --no-extras --slab-size 0 > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; return 1; }
  python3 -c "
import json; d = json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('$1 step', d['ms_per_step'], 'ms (graph)', 'eager', d.get('eager_ms_per_step'))" | tee -a $OUT/summary.txt
}
for rep in 1 2; do step nn.WINO_V_PREPASS=0 || exit 1; step nn.WINO_V_PREPASS=1 || exit 1; done
timeout -k 10 600 python -u scripts/r06/mod_ab.py nn.WINO_V_PREPASS=0 - > $OUT/slab.txt 2> $OUT/slab.err || { tail -20 $OUT/slab.err; exit 1; }
cat $OUT/slab.txt | tee -a $OUT/summary.txt
