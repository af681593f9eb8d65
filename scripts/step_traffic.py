"""HBM traffic of the whole training step by kernel, from two rocprofv3 passes
over the same `bench.py --no-extras` run: --pmc FETCH_SIZE and --pmc
WRITE_SIZE (each with --kernel-trace only).  FETCH_SIZE x2 on gfx950 (16-B
lane reads, MI355X_MICROARCH.md), WRITE_SIZE exact.  Dispatches are
serialised under --pmc, so the durations are standalone times.

usage: step_traffic.py FETCH_DIR WRITE_DIR STEPS [TOP]
Prints per kernel (summed over all dispatches / STEPS): GB read, GB written,
standalone ms and GB/s, then the totals per step.
"""
import csv
import sys
from collections import defaultdict


def load(d, counter):
    val, dur, name = defaultdict(float), {}, {}
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        if r.get("Counter_Name") != counter:
            continue
        k = int(r["Dispatch_Id"])
        val[k] += float(r["Counter_Value"])
        name[k] = r["Kernel_Name"].split("(")[0][:90]
        if r.get("End_Timestamp"):
            dur[k] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    if not dur:
        try:
            for r in csv.DictReader(open(f"{d}/run_kernel_trace.csv")):
                k = int(r["Dispatch_Id"])
                if k in name:
                    dur[k] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        except FileNotFoundError:
            pass
    return val, dur, name


def main():
    fd, wd, steps = sys.argv[1], sys.argv[2], int(sys.argv[3])
    top = int(sys.argv[4]) if len(sys.argv) > 4 else 30
    f, fdur, fname = load(fd, "FETCH_SIZE")
    w, _, wname = load(wd, "WRITE_SIZE")
    agg = defaultdict(lambda: [0.0, 0.0, 0.0, 0])
    for k, v in f.items():
        a = agg[fname[k]]
        a[0] += 2 * 1024 * v
        a[2] += fdur.get(k, 0)
        a[3] += 1
    for k, v in w.items():
        agg[wname[k]][1] += 1024 * v
    rows = sorted(agg.items(), key=lambda kv: -(kv[1][0] + kv[1][1]))
    tr = tw = tt = 0.0
    print(f"{'kernel':90s} {'rd GB':>7} {'wr GB':>7} {'ms':>7} {'GB/s':>6} {'n':>4}   (per step)")
    for n, (r, wb, t, c) in rows:
        tr += r
        tw += wb
        tt += t
        if top > 0:
            top -= 1
            gbs = (r + wb) / t if t else 0.0
            print(f"{n:90s} {r / steps / 1e9:7.3f} {wb / steps / 1e9:7.3f} {t / steps / 1e6:7.3f} {gbs:6.0f} "
                  f"{c // steps:4d}")
    print(f"TOTAL per step: read {tr / steps / 1e9:.2f} GB, write {tw / steps / 1e9:.2f} GB, "
          f"standalone kernel time {tt / steps / 1e6:.2f} ms, {(tr + tw) / tt if tt else 0:.0f} GB/s average")


if __name__ == "__main__":
    main()
