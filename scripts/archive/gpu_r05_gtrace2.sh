#!/bin/bash
# Kernel trace of the graph replay with the batched bias sums on (nn.BIAS_BATCHED=1),
# compared with r05graph5's (off) by scripts/graph_trace_cmp.py.
set -o pipefail
OUT=gpurun_out/${1:-r05gtrace2}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$OUT/tr -o run -- \
  python3 $GRAFT_REPO_ROOT/scripts/bench_ab.py nn.BIAS_BATCHED=1 -- --steps 6 --warmup 3 --no-extras --slab-size 0 > $GRAFT_REPO_ROOT/$OUT/tr.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$OUT/tr.log; exit 1; }
cd $GRAFT_REPO_ROOT
gzip -c $OUT/tr/run_kernel_trace.csv > $OUT/graph_kernel_trace.csv.gz && rm -rf $OUT/tr
tail -n 1 $OUT/tr.log | cut -c1-300
