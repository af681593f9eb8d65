#!/bin/bash
# Four interleaved chains in x3_gemm256_af_kernel (libm3d_quad.so: M3D_TUNE_X3_QUAD=1)
# vs the default build: parity tests on the quad build, then the priced launch and
# the step, same box.
set -o pipefail
OUT=gpurun_out/${1:-r05quad}
mkdir -p $OUT
export TMPDIR=/tmp
M3D_LIB_FILE=libm3d_quad.so timeout -k 10 500 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_configs.py tests/test_gpu_determinism.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -n 1 $OUT/pytest.log
for rep in 1 2; do
for lib in libm3d.so libm3d_quad.so; do
  timeout -k 10 120 env M3D_LIB_FILE=$lib python -u scripts/kernels_for_pmc.py gemm 128 > $OUT/k.json 2> $OUT/k.err || { tail -20 $OUT/k.err; exit 1; }
  python3 -c "
import ast; d = ast.literal_eval(open('$OUT/k.json').read().strip().splitlines()[-1]); print('$lib gemm', d['avg_launch_ms'], 'ms', d['achieved'], 'TF/s', d['frac'])" | tee -a $OUT/summary.txt
  timeout -k 10 240 env M3D_LIB_FILE=$lib python -u bench.py --steps 20 --warmup 3 --no-extras --slab-size 0 > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  python3 -c "
import json; d = json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('$lib step', d['ms_per_step'], 'ms (graph)', 'eager', d.get('eager_ms_per_step'))" | tee -a $OUT/summary.txt
done
done
