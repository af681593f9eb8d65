#!/bin/bash
# The graph-default tree: determinism (graph replay bitwise = eager), model and
# stream tests, then the bench line at its defaults without extras (graph) and --eager.
set -o pipefail
OUT=gpurun_out/${1:-r05graph6}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_determinism.py tests/test_gpu_streams.py tests/test_gpu_model.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -n 1 $OUT/pytest.log
for a in "" "--eager" "" "--eager"; do
  timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-extras $a > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  python3 -c "
import json; d = json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('[$a]', d['ms_per_step'], 'ms', d['value'], 'vol/s graph', d['config']['hip_graph'], 'eager', d.get('eager_ms_per_step'), d['config'].get('hip_graph_error'))"
done
