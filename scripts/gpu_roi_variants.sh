#!/bin/bash
# Usage: gpurun -- bash scripts/gpu_roi_variants.sh "V:SORT ..."   (M3D_ROI_VARIANT / M3D_ROI_SORT)
set -o pipefail
mkdir -p gpurun_out/roi_var
for spec in ${1:-0:1}; do
  IFS=: read v so <<< "$spec"
  M3D_ROI_VARIANT=$v M3D_ROI_SORT=$so timeout -k 10 120 python3 scripts/roi_variants.py > gpurun_out/roi_var/v${v}_$so.json 2> gpurun_out/roi_var/v${v}_$so.err || { tail -20 gpurun_out/roi_var/v${v}_$so.err; exit 1; }
  echo "sort=$so $(cat gpurun_out/roi_var/v${v}_$so.json)"
done
