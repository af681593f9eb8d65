set -o pipefail
mkdir -p gpurun_out/w2
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_conv.py -k "wgrad or winograd" > gpurun_out/w2/pt.log 2>&1 || { tail -40 gpurun_out/w2/pt.log; exit 1; }
tail -2 gpurun_out/w2/pt.log
for dbg in ${DBGS:-0}; do
  M3D_X3W_DBG=$dbg timeout -k 10 120 python -u scripts/kernels_for_pmc.py wgrad 128 > gpurun_out/w2/k.txt || exit 1
  python - $dbg <<'PY'
import ast, sys
d = ast.literal_eval(open("gpurun_out/w2/k.txt").read().strip().splitlines()[-1])
print("DBG", sys.argv[1], d["avg_launch_ms"], "ms", d["achieved"], "TF", d["frac"])
PY
done
