#!/bin/bash
# Winograd kernel profile A/B: rocprofv3 kernel stats of scripts/wino_prof.py under each env setting.
set -o pipefail
OUT=gpurun_out/${1:-wino_ab}
VARS=${2:-"M3D_WINO_GRAD4=0 M3D_WINO_GRAD4=1"}
mkdir -p $OUT
export TMPDIR=/tmp
for v in $VARS; do
  d=$OUT/$(echo $v | tr '=' '_')
  env $v timeout -k 10 300 rocprofv3 -f csv --kernel-trace --stats -d $d -o run -- python3 scripts/wino_prof.py > $d.log 2>&1 || { echo "$v failed"; tail -20 $d.log; exit 1; }
  rm -f $d/run_kernel_trace.csv
  echo "== $v"; python3 scripts/prof_summary.py $d/run_kernel_stats.csv 1 8
done
