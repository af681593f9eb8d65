set -o pipefail
mkdir -p gpurun_out/w2
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_gpu_conv.py -k "wgrad or winograd or conv_block" > gpurun_out/w2/pt.log 2>&1 || { tail -40 gpurun_out/w2/pt.log; exit 1; }
tail -3 gpurun_out/w2/pt.log
for tr in 1 0; do M3D_X3W_TR=$tr timeout -k 10 120 python -u scripts/kernels_for_pmc.py wgrad 128 || exit 1; done
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_gpu_model.py > gpurun_out/w2/pt2.log 2>&1 || { tail -40 gpurun_out/w2/pt2.log; exit 1; }
tail -3 gpurun_out/w2/pt2.log
