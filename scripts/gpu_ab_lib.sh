set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/ab2; mkdir -p $OUT
M3D_LIB_FILE=libm3d_ab.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_determinism.py -m gpu > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -n 1 $OUT/pytest.log
for rep in 1 2; do
for lib in libm3d.so libm3d_ab.so; do
  for leg in wgrad gemm; do
    M3D_LIB_FILE=$lib timeout -k 10 120 python -u scripts/kernels_for_pmc.py $leg 128 > $OUT/leg.txt 2>&1 || { tail -20 $OUT/leg.txt; exit 1; }
    python3 -c "
import ast; d = ast.literal_eval(open('$OUT/leg.txt').read().strip().splitlines()[-1])
print('$lib $leg', d['avg_launch_ms'], 'ms', d['achieved'], 'TF', d['frac'])"
  done
  M3D_LIB_FILE=$lib timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-extras --slab-size 0 > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  python3 -c "
import json; d = json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('$lib step', d['ms_per_step'], 'ms')"
done
done
