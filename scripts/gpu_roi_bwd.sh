set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/roi1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu -k "crop or pyramid or config2 or roi" > gpurun_out/roi1/pt.log 2>&1 || { tail -40 gpurun_out/roi1/pt.log; exit 1; }
tail -n 2 gpurun_out/roi1/pt.log
for g in 0 1; do for leg in roibwd7 roibwd14; do
  echo "== gather=$g $leg 128"; M3D_ROI_BWD_GATHER=$g timeout -k 10 120 python -u scripts/kernels_for_pmc.py $leg 128 2>&1 | tail -1
done; done
echo "== gather=1 roibwd14 256"; timeout -k 10 200 python -u scripts/kernels_for_pmc.py roibwd14 256 2>&1 | tail -1
echo "== gather=0 roibwd14 256"; M3D_ROI_BWD_GATHER=0 timeout -k 10 200 python -u scripts/kernels_for_pmc.py roibwd14 256 2>&1 | tail -1
