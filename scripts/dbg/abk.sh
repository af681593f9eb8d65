set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/abk; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_model.py tests/test_gpu_slab.py tests/test_gpu_determinism.py -m gpu > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -n 1 $OUT/pytest.log
for e in "M3D_CONV1_X3=1" "M3D_CONV1_X3=0"; do
  env $e timeout -k 10 200 python scripts/conv_layers.py --size 128 > $OUT/layers_$e.txt 2>&1 || exit 1
done
bash scripts/gpu_step_ab.sh abk "M3D_CONV1_X3=1" "M3D_CONV1_X3=0"
