#!/bin/bash
# tests + full bench + profiles at 128 and 256 + inference leg kernel stats
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r01e}
bash scripts/gpu_test_bench.sh $TAG || exit 1
bash scripts/gpu_prof.sh $TAG 128 || exit 1
LEGS="roi7:line_fwd_kernel:pyramid_fwd_pool7_S256_N512 roi14:line_fwd_kernel:pyramid_fwd_pool14_S256_N512" bash scripts/gpu_prof.sh ${TAG}_256 256 || exit 1
OUT=gpurun_out/$TAG
timeout -k 10 300 rocprofv3 -f csv --kernel-trace --stats -d $OUT/k_infer -o run -- python3 scripts/kernels_for_pmc.py infer 256 > $OUT/k_infer.log 2>&1 || { tail -20 $OUT/k_infer.log; exit 1; }
python3 scripts/prof_summary.py $OUT/k_infer/run_kernel_stats.csv 4 30 > $OUT/k_infer.txt
rm -f $OUT/k_infer/run_kernel_trace.csv
cat $OUT/k_infer.txt
