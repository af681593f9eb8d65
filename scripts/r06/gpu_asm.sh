#!/bin/bash
# x3_gemm256_af_kernel variants: per-step clock stamps (default / A 3-deep /
# asm loads), priced-launch times (default vs asm), parity of the asm build.
set -o pipefail
OUT=gpurun_out/${1:-r06asm}
mkdir -p $OUT
export TMPDIR=/tmp
for lib in libm3d_stamp.so libm3d_stampa3.so libm3d_stampasm.so; do
  echo "== $lib" >> $OUT/stamps.txt
  timeout -k 10 120 env M3D_LIB_FILE=$lib python -u scripts/r06/stamp_gemm.py 128 >> $OUT/stamps.txt 2>&1 || { tail -20 $OUT/stamps.txt; exit 1; }
done
cat $OUT/stamps.txt | grep -v amdgpu.ids
leg() {  # lib leg
  timeout -k 10 120 env M3D_LIB_FILE=$1 python -u scripts/kernels_for_pmc.py $2 128 > $OUT/k.json 2> $OUT/k.err || { tail -20 $OUT/k.err; return 1; }
  python3 -c "
import ast; d = ast.literal_eval(open('$OUT/k.json').read().strip().splitlines()[-1]); print('$1 $2', d['avg_launch_ms'], 'ms', d['achieved'], 'TF/s', d['frac'])" | tee -a $OUT/summary.txt
}
for rep in 1 2; do for lib in libm3d.so libm3d_asm.so; do leg $lib gemm || exit 1; done; done
timeout -k 10 900 env M3D_LIB_FILE=libm3d_asm.so python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_asm.log 2>&1 || { tail -30 $OUT/pytest_asm.log; exit 1; }
tail -n 2 $OUT/pytest_asm.log
step() {  # lib
  timeout -k 10 240 env M3D_LIB_FILE=$1 python -u bench.py --steps 20 --warmup 3 --no-extras --slab-size 0 > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; return 1; }
  python3 -c "
import json; d = json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('$1 step', d['ms_per_step'], 'ms (graph)', 'eager', d.get('eager_ms_per_step'))" | tee -a $OUT/summary.txt
}
for lib in libm3d.so libm3d_asm.so libm3d.so libm3d_asm.so; do step $lib || exit 1; done
