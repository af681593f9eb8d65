#!/bin/bash
# res2 branch2b (3^3, 64 -> 64) Winograd passes alone: HIP-event times and a
# rocprofv3 kernel-trace summary.  bash scripts/r06/gpu_res2prof.sh TAG
set -o pipefail
TAG=${1:-r06res2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 180 python -u scripts/r06/res2_prof.py > $OUT/times.txt 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/prof -o res2 -- python3 scripts/r06/res2_prof.py > $OUT/prof.log 2>&1
rc=$?
find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
echo rc=$rc
exit $rc
