#!/bin/bash
# Copy the judged summaries of a gpu_round2.sh run from gpurun_out/ into profiles/.
# Usage: bash scripts/archive_run.sh TAG   (reads gpurun_out/TAG and gpurun_out/TAG_256)
set -e
TAG=$1; O=gpurun_out/$TAG; O2=gpurun_out/${TAG}_256; P=profiles
cp $O/bench.json $P/${TAG}_bench_128.json
cp $O/pytest_gpu.log $P/${TAG}_pytest_gpu.log
[ -f $O/step_roofline_128.json ] && cp $O/step_roofline_128.json $P/${TAG}_step_roofline_128.json
[ -f $O/step_roofline_256.json ] && cp $O/step_roofline_256.json $P/${TAG}_step_roofline_256.json
[ -f $O/host_overhead.txt ] && cp $O/host_overhead.txt $P/${TAG}_host_overhead.txt
[ -f $O/smoke.log ] && cp $O/smoke.log $P/${TAG}_smoke.log
cp $O/bench_kernels.txt $P/${TAG}_bench_kernels_128.txt
cp $O/prof/run_kernel_stats.csv $P/${TAG}_bench_128_kernel_stats.csv
for leg in gemm wgrad direct roi7 roi14; do
  [ -f $O/k_$leg.txt ] && cp $O/k_$leg.txt $P/${TAG}_k_${leg}_128.txt && cp $O/k_$leg/run_kernel_stats.csv $P/${TAG}_k_${leg}_128_kernel_stats.csv
done
[ -f $O/k_infer.txt ] && cp $O/k_infer.txt $P/${TAG}_k_infer_256.txt && cp $O/k_infer/run_kernel_stats.csv $P/${TAG}_k_infer_256_kernel_stats.csv
if [ -d $O2 ]; then
  cp $O2/bench_kernels.txt $P/${TAG}_bench_kernels_256.txt
  cp $O2/prof/run_kernel_stats.csv $P/${TAG}_bench_256_kernel_stats.csv
  for leg in roi7 roi14; do
    [ -f $O2/k_$leg.txt ] && cp $O2/k_$leg.txt $P/${TAG}_k_${leg}_256.txt && cp $O2/k_$leg/run_kernel_stats.csv $P/${TAG}_k_${leg}_256_kernel_stats.csv
  done
fi
python3 - "$O/traffic.json" "$O2/traffic.json" <<'PY'
import json, os, sys
t = json.load(open("profiles/traffic.json")) if os.path.exists("profiles/traffic.json") else {}
for f in sys.argv[1:]:
    if os.path.exists(f):
        t.update(json.load(open(f)))
json.dump(t, open("profiles/traffic.json", "w"), indent=1, sort_keys=True)
PY
