#!/bin/bash
# One gpurun call: GPU parity tests, bench line, rocprofv3 kernel stats of the
# bench and separate FETCH_SIZE / WRITE_SIZE PMC passes of the dominant kernels.
# Usage (from repo root): gpurun --timeout 1200 -- bash scripts/gpu_full.sh TAG
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 420 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-extras > $OUT/prof_bench.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof_bench.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_kern -o run -- python3 scripts/kernels_for_pmc.py > $OUT/prof_kern.log 2>&1 || { echo "rocprof kern failed"; tail -30 $OUT/prof_kern.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_fetch -o run -- python3 scripts/kernels_for_pmc.py > $OUT/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; tail -30 $OUT/pmc_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/pmc_write -o run -- python3 scripts/kernels_for_pmc.py > $OUT/pmc_write.log 2>&1 || { echo "pmc write failed"; tail -30 $OUT/pmc_write.log; exit 1; }
find $OUT -name "*.csv" | head -20
echo DONE
