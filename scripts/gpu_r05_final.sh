#!/bin/bash
# Round-5 evidence on one box: all -m gpu tests, smoke(), the full bench line
# (step-roofline tables), then rocprofv3 kernel stats of the 128^3 step and the
# priced launches with separate FETCH_SIZE / WRITE_SIZE passes (gpu_prof.sh).
# Usage: gpurun --timeout 1200 -- bash scripts/gpu_r05_final.sh TAG
set -o pipefail
TAG=${1:-r05final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -n 1 $OUT/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -n 1 $OUT/smoke.log
M3D_STEP_ROOFLINE_TABLE=$OUT/step_roofline_128.json M3D_STEP_ROOFLINE_TABLE_256=$OUT/step_roofline_256.json \
  timeout -k 10 500 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print(json.dumps(d['summary']))"
LEGS="wgrad:x3_wgrad:wino_wgrad_gemm_rpn_shared1_S128 gemm:x3_gemm256_af_kernel:wino_gemm_x3af_rpn_shared1_S128" bash scripts/gpu_prof.sh $TAG 128 > $OUT/prof128.log 2>&1 || { echo "prof 128 failed"; tail -20 $OUT/prof128.log; exit 1; }
head -14 $OUT/bench_kernels.txt
echo DONE
