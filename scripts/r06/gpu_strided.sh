#!/bin/bash
# (2,2,1)-strided 1x1x1 weight gradients as subsample + split GEMM: conv tests,
# then same-box A/Bs (nn.WGRAD1_STRIDED_X3 0 / 1) at 128^3 and 256^3.
set -o pipefail
OUT=gpurun_out/${1:-r06str}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_conv.py -k "conv_block_fwd_bwd" tests/test_gpu_bnfuse.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
grep -c PASSED $OUT/tests.log
step() {
  timeout -k 10 240 python -u scripts/bench_ab.py $1 -- --steps 20 --warmup 3 --no-extras --slab-size 0 > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; return 1; }
  python3 -c "
import json; d = json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('$1 step', d['ms_per_step'], 'ms (graph)', 'eager', d.get('eager_ms_per_step'))" | tee -a $OUT/summary.txt
}
for rep in 1 2; do step nn.WGRAD1_STRIDED_X3=0 || exit 1; step nn.WGRAD1_STRIDED_X3=1 || exit 1; done
timeout -k 10 600 python -u scripts/r06/mod_ab.py nn.WGRAD1_STRIDED_X3=0 - > $OUT/slab.txt 2> $OUT/slab.err || { tail -20 $OUT/slab.err; exit 1; }
cat $OUT/slab.txt | tee -a $OUT/summary.txt
