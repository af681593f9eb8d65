#!/bin/bash
# Round-end evidence: smoke, all GPU tests, the default bench line, 128^3 and
# 256^3 kernel stats + PMC traffic of the priced launches, inference kernel stats.
# Usage (repo root): gpurun --timeout 1200 -- bash scripts/gpu_final.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r01t}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
bash scripts/gpu_round2.sh $TAG
