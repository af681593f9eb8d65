#!/bin/bash
# spill-free x3_gemm256_af_kernel<2>: fused-BN parity tests, then same-box
# A/Bs of nn.X3_BN_FUSE at 128^3 (graph step) and 256^3.  bash scripts/r06/gpu_fuse.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-r06fuse}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_bnfuse.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
grep -c PASSED $OUT/tests.log
step() {
  timeout -k 10 240 python -u scripts/bench_ab.py nn.X3_BN_FUSE=$1 -- --steps 20 --warmup 3 --no-extras --slab-size 0 > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; return 1; }
  python3 -c "
import json; d = json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('X3_BN_FUSE=$1 step', d['ms_per_step'], 'ms (graph)', 'eager', d.get('eager_ms_per_step'))" | tee -a $OUT/summary.txt
}
for rep in 1 2; do for f in 0 1; do step $f || exit 1; done; done
timeout -k 10 500 python -u scripts/r06/fuse_ab.py > $OUT/slab.txt 2> $OUT/slab.err || { tail -20 $OUT/slab.err; exit 1; }
cat $OUT/slab.txt | tee -a $OUT/summary.txt
