#!/bin/bash
# One-step kernel trace: per-dispatch Winograd transform bandwidth.
set -o pipefail
O=gpurun_out/trace_w; mkdir -p $O
export TMPDIR=/tmp
M3D_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 -f csv --kernel-trace -d $O/t -o run -- python3 bench.py --steps 1 --warmup 1 --no-extras --no-proposals > $O/log 2>&1 || { tail -20 $O/log; exit 1; }
python3 - $O/t/run_kernel_trace.csv <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
last = {}
for name, per in (("wino_input_kernel<4>", 44), ("wino_output_kernel<4>", 44), ("wino_grad_kernel<2>", 22), ("wino_input_kernel<2>", 22)):
    rs = [r for r in rows if name in r["Kernel_Name"]][-per:]
    tot_t = tot_b = 0
    for r in rs:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        TC = int(r["Grid_Size_X"])
        pts = 96 if "<4>" in name else 64
        out_per = 16 if "<4>" in name else 8
        b = 4.0 * TC * (pts + out_per)
        tot_t += d; tot_b += b
    big = sorted(rs, key=lambda r: -int(r["Grid_Size_X"]))[:3]
    print(f"{name}: {len(rs)} launches {tot_t*1e3:.2f} ms, {tot_b/1e9:.2f} GB -> {tot_b/tot_t/1e12:.2f} TB/s;",
          " biggest:", [(int(r['Grid_Size_X']), round((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3,1)) for r in big])
PY
