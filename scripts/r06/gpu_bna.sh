#!/bin/bash
# identity-block 2a data gradients on the split GEMM with the fused BN-ReLU
# backward and accumulate (m3d_conv3d_bwd_data_x3_bna): fused-BN tests, then
# same-box A/Bs against the previous routing at 128^3 and 256^3.
set -o pipefail
OUT=gpurun_out/${1:-r06bna}
mkdir -p $OUT
export TMPDIR=/tmp
A=nn.CONV1_X3_DGRAD_FUSED_MIN_K=256,nn.X3_BN_FUSE_ACC=0
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_bnfuse.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
grep -c PASSED $OUT/tests.log
step() {
  timeout -k 10 240 python -u scripts/bench_ab.py $1 -- --steps 20 --warmup 3 --no-extras --slab-size 0 > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; return 1; }
  python3 -c "
import json; d = json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('$1 step', d['ms_per_step'], 'ms (graph)', 'eager', d.get('eager_ms_per_step'))" | tee -a $OUT/summary.txt
}
for rep in 1 2; do step $A || exit 1; step nn.X3_BN_FUSE_ACC=1 || exit 1; done
timeout -k 10 600 python -u scripts/r06/mod_ab.py $A - > $OUT/slab.txt 2> $OUT/slab.err || { tail -20 $OUT/slab.err; exit 1; }
cat $OUT/slab.txt | tee -a $OUT/summary.txt
