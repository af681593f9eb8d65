#!/bin/bash
# rocprofv3 kernel stats of the 128^3 step + the priced launches' PMC traffic,
# then the 256^3 ROIAlign legs.  bash scripts/r06/gpu_prof_final.sh TAG
set -o pipefail
TAG=${1:-r06prof}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
bash scripts/gpu_prof.sh $TAG 128 > $OUT/prof128.log 2>&1 || { echo "prof 128 failed"; tail -20 $OUT/prof128.log; exit 1; }
LEGS="roi7:line_fwd_sl_kernel:pyramid_fwd_pool7_S256_N512 roi14:line_fwd_sl_kernel:pyramid_fwd_pool14_S256_N512" bash scripts/gpu_prof.sh ${TAG}_256 256 > $OUT/prof256.log 2>&1 || { echo "prof 256 failed"; tail -20 $OUT/prof256.log; exit 1; }
head -12 $OUT/bench_kernels.txt
echo DONE
