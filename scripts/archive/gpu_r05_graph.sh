#!/bin/bash
# HIP-graph replay vs eager: the replayed step under the
# runtime's graph-execution modes (r05graph: packet capture off and a forced
# count of graph streams changed nothing) and with more hardware queues per
# process (HWQ), so the replay's parallel branches stop sharing a queue with
# the weight-gradient backlog.
set -o pipefail
OUT=gpurun_out/${1:-r05graph}
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # label, env assignment, bench args
  local label=$1 envs=$2; shift 2
  timeout -k 10 240 env $envs python -u bench.py --steps 20 --warmup 3 --no-extras --slab-size 0 "$@" > $OUT/b.json 2> $OUT/b_$label.err || { tail -20 $OUT/b_$label.err; exit 1; }
  python3 -c "
import json; d = json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('$label', 'step', d['ms_per_step'], 'ms', d['value'], 'vol/s')" | tee -a $OUT/summary.txt
}
for rep in 1 2; do
  run eager M3D_X=0
  run graph M3D_X=0 --graph
  for q in ${HWQ:-8 16}; do
    run eager_hwq$q GPU_MAX_HW_QUEUES=$q
    run graph_hwq$q GPU_MAX_HW_QUEUES=$q --graph
  done
done
