#!/bin/bash
# 256^3 depth-slab step (N=1) A/B of the 1x1x1 split-GEMM selection, same box:
# round-5 default vs round-4 data-gradient rule (K >= 256) vs round-4 rules both ways.
set -o pipefail
OUT=gpurun_out/${1:-r05slab}
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
for sw in nn.CONV1_X3_MIN_K=32 nn.CONV1_X3_DGRAD_MIN_K=256 nn.CONV1_X3_DGRAD_MIN_K=256,nn.CONV1_X3_MIN_K=256,nn.CONV1_X3_FWD_TILES=256; do
  timeout -k 10 300 python -u scripts/slab_leg.py 256 $sw > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  echo "$sw $(tail -n 1 $OUT/b.json)" | tee -a $OUT/summary.txt
done
done
