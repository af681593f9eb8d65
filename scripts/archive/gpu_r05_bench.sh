#!/bin/bash
# The bench line at its defaults (what the driver runs), one JSON line kept.
set -o pipefail
OUT=gpurun_out/${1:-r05bench}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); r=d['roofline']; print(d['value'], d['ms_per_step'], d.get('eager_ms_per_step'), r['kernel'][:40], r['avg_launch_ms'], r['frac'], r['traffic'], r['wgrad_gemm']['avg_launch_ms'], r['wgrad_gemm']['frac'], json.dumps(d.get('summary')))"
