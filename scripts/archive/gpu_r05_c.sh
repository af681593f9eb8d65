#!/bin/bash
# GPU suite + gradient error table (base host variants) + a short 128^3 bench
# of the current tree.  Usage: gpurun -- bash scripts/archive/gpu_r05_c.sh TAG
set -o pipefail
TAG=${1:-r05c}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -n 2 $OUT/pytest_gpu.log
grep "gradients:" $OUT/pytest_gpu.log || true
timeout -k 10 300 python -u scripts/grad_table.py --out $OUT/grad.json --variants base > $OUT/grad.log 2>&1 || { tail -30 $OUT/grad.log; exit 1; }
grep median $OUT/grad.log | cut -c1-300
timeout -k 10 200 python -u bench.py --steps 10 --warmup 5 --no-extras > $OUT/bench128.log 2>&1 || { tail -30 $OUT/bench128.log; exit 1; }
tail -c 600 $OUT/bench128.log
