#!/bin/bash
# PyramidROIAlign forward variants A/B (one process per variant).
set -o pipefail
OUT=gpurun_out/${1:-roi_ab}
VARS=${2:-"M3D_ROI_SLICES=1 M3D_ROI_SLICES=2 M3D_ROI_SLICES=4 M3D_ROI_SLICES=8"}
mkdir -p $OUT
for v in $VARS; do
  env $v timeout -k 10 300 python -u scripts/roi_ab.py >> $OUT/roi_ab.jsonl 2>> $OUT/roi_ab.err || { echo "$v failed"; tail -20 $OUT/roi_ab.err; exit 1; }
done
cat $OUT/roi_ab.jsonl
