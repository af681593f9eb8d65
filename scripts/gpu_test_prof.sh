#!/bin/bash
# rocprofv3 kernel stats of the 128^3 bench step (after optional GPU tests + bench line).
# Usage: gpurun -- bash scripts/gpu_test_prof.sh TAG [notest]
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$2" != "notest" ]; then bash scripts/gpu_test_bench.sh $TAG || exit 1; fi
timeout -k 10 300 rocprofv3 -f csv --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-extras > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
python3 scripts/prof_summary.py $OUT/prof/run_kernel_stats.csv 7 30 > $OUT/bench_kernels.txt
rm -f $OUT/prof/run_kernel_trace.csv
cat $OUT/bench_kernels.txt
