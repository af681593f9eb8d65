#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-r06asm2}
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # lib
  timeout -k 10 240 env M3D_LIB_FILE=$1 python -u bench.py --steps 20 --warmup 3 --no-extras --slab-size 0 > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; return 1; }
  python3 -c "
import json; d = json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('$1 step', d['ms_per_step'], 'ms (graph)', 'eager', d.get('eager_ms_per_step'))" | tee -a $OUT/summary.txt
}
for lib in libm3d.so libm3d_asm.so; do step $lib || exit 1; done
for lib in libm3d.so libm3d_asm.so; do
  timeout -k 10 400 env M3D_LIB_FILE=$lib python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q -k "atomic_and_256" --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_$lib.log 2>&1; echo "$lib rc=$?" | tee -a $OUT/summary.txt
  grep "gradients:" $OUT/pytest_$lib.log | cut -c1-200 | tee -a $OUT/summary.txt
done
