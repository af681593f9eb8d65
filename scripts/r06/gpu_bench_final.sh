#!/bin/bash
# the full bench line with the step-roofline tables (128^3, 256^3)
set -o pipefail
TAG=${1:-r06final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
M3D_STEP_ROOFLINE_TABLE=$OUT/step_roofline_128.json M3D_STEP_ROOFLINE_TABLE_256=$OUT/step_roofline_256.json \
  timeout -k 10 1000 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d.get('eager_ms_per_step'), json.dumps(d.get('summary')))"
