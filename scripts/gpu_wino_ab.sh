#!/bin/bash
# GPU tests (default: F(2x2x4) fwd/dgrad, F(2x2x2) wgrad) + bench step time for
# Winograd tile configs (M3D_WINO_NZ / M3D_WINO_WGRAD_NZ) + conv layer table.
set -o pipefail
O=gpurun_out/wab; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cfg in "4 2" "2 2" "4 4"; do
  set -- $cfg
  M3D_WINO_NZ=$1 M3D_WINO_WGRAD_NZ=$2 timeout -k 10 300 python3 bench.py --no-extras --slab-size 0 > $O/bench_$1$2.json 2> $O/bench_$1$2.err || { tail -20 $O/bench_$1$2.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$1$2.json')); print('NZ=$1 WGRAD_NZ=$2 step ms', d['ms_per_step'], 'vol/s', d['value'])"
done
M3D_WINO_NZ=4 M3D_WINO_WGRAD_NZ=4 timeout -k 10 300 python -m pytest tests/test_gpu_model.py -q -k backward > $O/pytest44.log 2>&1; grep -o "assert 0.000[0-9]* < 0.0001" $O/pytest44.log | head -2
timeout -k 10 300 python3 scripts/conv_bench.py > $O/conv.txt 2>&1 || { tail -20 $O/conv.txt; exit 1; }
grep -v amdgpu $O/conv.txt
