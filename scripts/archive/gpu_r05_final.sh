#!/bin/bash
# Round-5 evidence, call A: all -m gpu tests, smoke(), the full bench line
# (with the step-roofline tables).  Call B: scripts/archive/gpu_r05_prof.sh.
# Usage: gpurun --timeout 1200 -- bash scripts/archive/gpu_r05_final.sh TAG
set -o pipefail
TAG=${1:-r05final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -rA > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -n 1 $OUT/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -n 1 $OUT/smoke.log
M3D_STEP_ROOFLINE_TABLE=$OUT/step_roofline_128.json M3D_STEP_ROOFLINE_TABLE_256=$OUT/step_roofline_256.json \
  timeout -k 10 500 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d.get('eager_ms_per_step'), json.dumps(d.get('summary')))"
echo DONE
