#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-r05conv1}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/conv1_paths.py > $OUT/conv1_paths.txt 2>&1 || { tail -20 $OUT/conv1_paths.txt; exit 1; }
cat $OUT/conv1_paths.txt
