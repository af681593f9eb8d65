#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-r06a3}
mkdir -p $OUT
export TMPDIR=/tmp
leg() {  # lib leg
  timeout -k 10 120 env M3D_LIB_FILE=$1 python -u scripts/kernels_for_pmc.py $2 128 > $OUT/k.json 2> $OUT/k.err || { tail -20 $OUT/k.err; return 1; }
  python3 -c "
import ast; d = ast.literal_eval(open('$OUT/k.json').read().strip().splitlines()[-1]); print('$1 $2', d['avg_launch_ms'], 'ms', d['achieved'], 'TF/s', d['frac'])" | tee -a $OUT/summary.txt
}
step() {  # lib
  timeout -k 10 240 env M3D_LIB_FILE=$1 python -u bench.py --steps 20 --warmup 3 --no-extras --slab-size 0 > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; return 1; }
  python3 -c "
import json; d = json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('$1 step', d['ms_per_step'], 'ms (graph)', 'eager', d.get('eager_ms_per_step'))" | tee -a $OUT/summary.txt
}
for rep in 1 2; do for lib in libm3d.so libm3d_a3.so; do leg $lib gemm || exit 1; done; done
for lib in libm3d.so libm3d_a3.so libm3d.so libm3d_a3.so; do step $lib || exit 1; done
timeout -k 10 600 env M3D_LIB_FILE=libm3d_a3.so python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_conv.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_a3.log 2>&1; echo "a3 tests rc=$?" | tee -a $OUT/summary.txt
tail -n 2 $OUT/pytest_a3.log
