#!/bin/bash
# HIP-graph replay vs eager with the weight gradient enqueued after the data
# gradient (nn.WGRAD_LAST): does the capture order decide which of the
# replay's streams the compute-path nodes land on?  Plus a kernel trace of the
# graph replay in that order (scripts/graph_trace_cmp.py).
set -o pipefail
OUT=gpurun_out/${1:-r05graph3}
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # label, module switches, bench args
  local label=$1 sw=$2; shift 2
  timeout -k 10 240 python -u scripts/bench_ab.py "$sw" -- --steps 20 --warmup 3 --no-extras --slab-size 0 "$@" > $OUT/b.json 2> $OUT/b_$label.err || { tail -20 $OUT/b_$label.err; exit 1; }
  python3 -c "
import json; d = json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('$label', 'step', d['ms_per_step'], 'ms', d['value'], 'vol/s')" | tee -a $OUT/summary.txt
}
for rep in 1 2; do
  run eager nn.WGRAD_LAST=0
  run eager_wlast_pal nn.WGRAD_LAST=1,model.PROPOSALS_AFTER_LOSS=1
  run graph_wlast nn.WGRAD_LAST=1 --graph
  run graph_wlast_pal nn.WGRAD_LAST=1,model.PROPOSALS_AFTER_LOSS=1 --graph
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$OUT/tr -o run -- \
  python3 $GRAFT_REPO_ROOT/scripts/bench_ab.py nn.WGRAD_LAST=1,model.PROPOSALS_AFTER_LOSS=1 -- --steps 6 --warmup 3 --no-extras --slab-size 0 --graph > $GRAFT_REPO_ROOT/$OUT/tr.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$OUT/tr.log; exit 1; }
cd $GRAFT_REPO_ROOT
gzip -c $OUT/tr/run_kernel_trace.csv > $OUT/graph_kernel_trace.csv.gz && rm -rf $OUT/tr
echo DONE
