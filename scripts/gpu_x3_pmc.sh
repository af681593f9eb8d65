#!/bin/bash
# SQ counters of the X3 Winograd point GEMM vs the f32 one (winofwd leg).
set -o pipefail
for x in 1 0; do
  M3D_GEMM_X3=$x bash scripts/gpu_pmc_sq.sh winofwd 128 "${KS:-gemm_kernel}" x3pmc$x || exit 1
done
