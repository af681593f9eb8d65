#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-r06pretest}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wino_prepass.py tests/test_gpu_determinism.py tests/test_gpu_config0.py tests/test_gpu_configs.py tests/test_gpu_bnfuse.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
