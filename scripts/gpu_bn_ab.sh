#!/bin/bash
# A/B of the bn_act_bwd grid size (M3D_BN_BLOCKS): per-step kernel time + bench ms/step.
set -o pipefail
O=gpurun_out/bn_ab; mkdir -p $O
export TMPDIR=/tmp
for nb in ${@:-512 2048 4096}; do
  M3D_BN_BLOCKS=$nb M3D_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 -f csv --kernel-trace -d $O/t$nb -o run -- python3 bench.py --steps 1 --warmup 1 --no-extras --no-proposals > $O/log$nb 2>&1 || { tail -20 $O/log$nb; exit 1; }
  echo "== M3D_BN_BLOCKS=$nb"; python3 scripts/trace_top.py $O/t$nb/run_kernel_trace.csv bn_act_bwd_kernel 76 | tail -1
  python3 scripts/trace_top.py $O/t$nb/run_kernel_trace.csv bn_sums_reduce 76 | tail -1
  rm -f $O/t$nb/run_kernel_trace.csv
  M3D_BN_BLOCKS=$nb timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-extras > $O/b$nb 2>&1 || exit 1
  grep -o '"ms_per_step": [0-9.]*' $O/b$nb
done
