#!/bin/bash
# Round-5 evidence, call B: rocprofv3 kernel stats of the 128^3 eager step and
# of the priced launches with FETCH_SIZE / WRITE_SIZE passes (gpu_prof.sh),
# then the kernel table of the configs[3] inference pass at 256^3.
set -o pipefail
TAG=${1:-r05prof}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
LEGS="wgrad:x3_wgrad:wino_wgrad_gemm_rpn_shared1_S128 gemm:x3_gemm256_af_kernel:wino_gemm_x3af_rpn_shared1_S128" bash scripts/gpu_prof.sh $TAG 128 > $OUT/prof128.log 2>&1 || { echo "prof 128 failed"; tail -20 $OUT/prof128.log; exit 1; }
head -14 $OUT/bench_kernels.txt
timeout -k 10 300 rocprofv3 -f csv --kernel-trace --stats -d $OUT/k_infer -o run -- python3 scripts/kernels_for_pmc.py infer 256 > $OUT/k_infer.log 2>&1 || { echo "infer prof failed"; tail -20 $OUT/k_infer.log; exit 1; }
python3 scripts/prof_summary.py $OUT/k_infer/run_kernel_stats.csv 4 30 > $OUT/k_infer_256.txt
rm -f $OUT/k_infer/run_kernel_trace.csv
head -8 $OUT/k_infer_256.txt
echo DONE
