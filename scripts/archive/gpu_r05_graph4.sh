#!/bin/bash
# Host cost of the HIP-graph replay vs the eager enqueue (scripts/host_overhead.py --graph).
set -o pipefail
OUT=gpurun_out/${1:-r05graph4}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/host_overhead.py --graph --no-profile > $OUT/host_graph.txt 2>&1 || { tail -20 $OUT/host_graph.txt; exit 1; }
timeout -k 10 300 python -u scripts/host_overhead.py --graph --wgrad-last --no-profile > $OUT/host_graph_wlast.txt 2>&1 || { tail -20 $OUT/host_graph_wlast.txt; exit 1; }
grep -h "host\|graph" $OUT/host_graph.txt $OUT/host_graph_wlast.txt
