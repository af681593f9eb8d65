#!/bin/bash
# GPU tests (conv + model) + one bench line + the step's kernel stats.  Usage: gpu_quick_prof.sh TAG
set -o pipefail
TAG=${1:-q}; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_conv.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-extras > $O/b.json 2>&1 || { tail -5 $O/b.json; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $O/b.json
timeout -k 10 300 rocprofv3 -f csv --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-extras > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/prof_summary.py $O/prof/run_kernel_stats.csv 7 40 > $O/kernels.txt
rm -f $O/prof/run_kernel_trace.csv
cat $O/kernels.txt
