#!/bin/bash
# One-step kernel trace of the 128^3 bench step; per-dispatch tables of the main kernels.
set -o pipefail
O=gpurun_out/trace; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 -f csv --kernel-trace -d $O/t -o run -- python3 bench.py --steps 1 --warmup 1 --no-extras > $O/log 2>&1 || { tail -20 $O/log; exit 1; }
python3 scripts/trace_top.py $O/t/run_kernel_trace.csv conv_wgrad_kernel 75 > $O/wgrad.txt
python3 scripts/trace_top.py $O/t/run_kernel_trace.csv "conv_gemm_kernel" 140 > $O/gemm.txt
python3 scripts/trace_top.py $O/t/run_kernel_trace.csv "bn_act_bwd_kernel" 76 > $O/bnbwd.txt
gzip -f $O/t/run_kernel_trace.csv
head -45 $O/wgrad.txt; tail -1 $O/wgrad.txt; head -30 $O/gemm.txt; tail -1 $O/gemm.txt; head -12 $O/bnbwd.txt; tail -1 $O/bnbwd.txt
