#!/bin/bash
# Re-entry check on the rebuilt tree: all -m gpu tests, smoke(), the bench line.
set -o pipefail
OUT=gpurun_out/r03z2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -n 1 $OUT/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -n 1 $OUT/smoke.log
timeout -k 10 500 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
tail -n 1 $OUT/bench.json
echo DONE
