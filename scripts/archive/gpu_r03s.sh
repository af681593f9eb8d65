#!/bin/bash
# 256^3 allocator fixes (throttle) + step A/B of the x3 weight gradient for the Cout=64 1x1x1 convs
set -o pipefail
bash scripts/archive/gpu_r03r.sh || exit 1
bash scripts/gpu_step_ab.sh r03s/ab "M3D_WGRAD1_X3_MIN_N=65" "M3D_WGRAD1_X3_MIN_N=64" || true
