#!/bin/bash
# A/B: libm3d with non-temporal Winograd transform streams (in tree) vs without (m3d/libm3d_t.so)
set -o pipefail
O=gpurun_out/nt; mkdir -p $O
timeout -k 10 300 python -m pytest tests -m gpu -x -q -k "wino or conv or model" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
timeout -k 10 300 python3 bench.py --no-extras --slab-size 0 > $O/b.json 2>/dev/null || exit 1
python3 -c "import json; d=json.load(open('$O/b.json')); print('NT step ms', d['ms_per_step'])"
cp 3d-mask-r-cnn_amd/m3d/libm3d.so $O/keep.so && cp 3d-mask-r-cnn_amd/m3d/libm3d_t.so 3d-mask-r-cnn_amd/m3d/libm3d.so
timeout -k 10 300 python3 bench.py --no-extras --slab-size 0 > $O/b.json 2>/dev/null || exit 1
python3 -c "import json; d=json.load(open('$O/b.json')); print('T  step ms', d['ms_per_step'])"
cp $O/keep.so 3d-mask-r-cnn_amd/m3d/libm3d.so
done
