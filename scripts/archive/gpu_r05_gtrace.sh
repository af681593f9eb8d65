#!/bin/bash
# Kernel traces of the eager and the HIP-graph-replayed 128^3 step (VERDICT r4
# item 5): per-kernel durations, queues and gaps compared offline
# (scripts/graph_trace_cmp.py).
set -o pipefail
OUT=gpurun_out/${1:-r05gtrace}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for mode in eager graph; do
  arg=""; [ $mode = graph ] && arg="--graph"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$OUT/$mode -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 3 --no-extras --slab-size 0 $arg > $GRAFT_REPO_ROOT/$OUT/$mode.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$OUT/$mode.log; exit 1; }
  tail -n 1 $GRAFT_REPO_ROOT/$OUT/$mode.log | cut -c1-200
done
cd $GRAFT_REPO_ROOT
for mode in eager graph; do
  f=$(ls $OUT/$mode/*/*kernel_trace.csv $OUT/$mode/*kernel_trace.csv 2>/dev/null | head -n 1)
  gzip -c "$f" > $OUT/${mode}_kernel_trace.csv.gz && ls -la $OUT/${mode}_kernel_trace.csv.gz
done
rm -rf $OUT/eager $OUT/graph
