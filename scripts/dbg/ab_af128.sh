set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/af128; mkdir -p $OUT
M3D_X3_AF128=0 timeout -k 10 120 python scripts/dbg/af128_check.py $OUT/c0.npy 2>&1 | grep -v amdgpu.ids || exit 1
M3D_X3_AF128=1 timeout -k 10 120 python scripts/dbg/af128_check.py $OUT/c1.npy 2>&1 | grep -v amdgpu.ids || exit 1
python3 -c "import numpy as np; a=np.load('$OUT/c0.npy'); b=np.load('$OUT/c1.npy'); print('bitwise equal:', np.array_equal(a.view(np.uint32), b.view(np.uint32)))"
for e in M3D_X3_AF128=0 M3D_X3_AF128=1 M3D_X3_AF128=0 M3D_X3_AF128=1; do
  env $e timeout -k 10 120 python -u scripts/kernels_for_pmc.py gemm 128 > $OUT/leg.txt 2>&1 || { tail -5 $OUT/leg.txt; exit 1; }
  python3 -c "
import ast; d = ast.literal_eval(open('$OUT/leg.txt').read().strip().splitlines()[-1]); print('$e leg', d['avg_launch_ms'], 'ms', d['achieved'], 'TF', d['frac'])"
done
bash scripts/gpu_step_ab.sh af128 "M3D_X3_AF128=0" "M3D_X3_AF128=1"
