#!/bin/bash
# Round-end evidence on one box: all -m gpu tests, smoke(), the full bench line,
# rocprofv3 kernel stats of the 128^3 / 256^3 steps and the priced launches
# (+ PMC traffic passes).  Usage: gpurun --timeout 1200 -- bash scripts/gpu_final.sh TAG
set -o pipefail
TAG=${1:-r02i}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -n 1 $OUT/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -n 1 $OUT/smoke.log
M3D_STEP_ROOFLINE_TABLE=$OUT/step_roofline_128.json M3D_STEP_ROOFLINE_TABLE_256=$OUT/step_roofline_256.json \
  timeout -k 10 500 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
timeout -k 10 200 python scripts/host_overhead.py > $OUT/host_overhead.txt 2>&1 || { echo "host overhead failed"; tail -20 $OUT/host_overhead.txt; exit 1; }
cat $OUT/host_overhead.txt
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['depth_slab']['ms_per_step'])"
bash scripts/gpu_prof.sh $TAG 128 > $OUT/prof128.log 2>&1 || { echo "prof 128 failed"; tail -20 $OUT/prof128.log; exit 1; }
LEGS="roi7:line_fwd_sl_kernel:pyramid_fwd_pool7_S256_N512 roi14:line_fwd_sl_kernel:pyramid_fwd_pool14_S256_N512" bash scripts/gpu_prof.sh ${TAG}_256 256 > $OUT/prof256.log 2>&1 || { echo "prof 256 failed"; tail -20 $OUT/prof256.log; exit 1; }
head -12 $OUT/bench_kernels.txt
echo DONE
