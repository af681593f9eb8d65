#!/bin/bash
# 64-channel Winograd kernels (x3_wgrad64_kernel, x3_gemm_kernel<..., 64>):
# parity tests, res2 layers alone, and same-box step A/Bs (128^3 graph step,
# 256^3 depth-slab step) against the previous library.  bash scripts/r06/gpu_c64.sh TAG
set -o pipefail
TAG=${1:-r06c64}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
P=res2a_branch2b+res2b_branch2b+res2c_branch2b
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_conv.py \
  -k "split3_exact_and_gemm_x3 or wino_weight_gradient_accuracy or conv_block_fwd_bwd or batched_wgrad_gemm" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_determinism.py \
  -k "weight_gradient_bitwise" >> $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
grep -c PASSED $OUT/tests.log
for lib in libm3d_prev.so libm3d.so; do
  M3D_LIB_FILE=$lib timeout -k 10 180 python -u scripts/r06/res2_prof.py > $OUT/res2_$lib.txt 2>&1 || { tail $OUT/res2_$lib.txt; exit 1; }
  echo "$lib $(grep res2_256 $OUT/res2_$lib.txt | head -1)" | tee -a $OUT/summary.txt
done
step() {
  timeout -k 10 240 env M3D_LIB_FILE=$1 python -u bench.py --steps 20 --warmup 3 --no-extras --slab-size 0 > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; return 1; }
  python3 -c "
import json; d = json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('$1 step', d['ms_per_step'], 'ms (graph)', 'eager', d.get('eager_ms_per_step'))" | tee -a $OUT/summary.txt
}
for rep in 1 2; do for lib in libm3d_prev.so libm3d.so; do step $lib || exit 1; done; done
for lib in libm3d_prev.so libm3d.so; do
  M3D_LIB_FILE=$lib timeout -k 10 400 python -u scripts/r06/slab_ab.py $P > $OUT/slab_$lib.txt 2> $OUT/slab.err || { tail -20 $OUT/slab.err; exit 1; }
  echo "$lib 256 $(cat $OUT/slab_$lib.txt | tr '\n' ' ')" | tee -a $OUT/summary.txt
done
