"""Compare rocprofv3 kernel traces of the eager and the HIP-graph-replayed
training step (scripts/archive/gpu_r05_gtrace.sh): per step, the span, the summed
kernel time, the union of busy time, the queues kernels landed on and the
kernel groups whose time differs most.  Steps are delimited by the optimizer's
sgd_update_kernel (one per step, after the backward)."""
import collections
import csv
import gzip
import sys


def load(path):
    rows = list(csv.DictReader(gzip.open(path, "rt")))
    for r in rows:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        r["q"] = r["Queue_Id"]
        r["n"] = r["Kernel_Name"].split("(")[0].replace("void ", "")[:70]
    rows.sort(key=lambda r: r["s"])
    return rows


def steps(rows, last=4):
    ends = [r["e"] for r in rows if "sgd_update_kernel" in r["n"]]
    out = []
    for a, b in zip(ends[-last - 1:-1], ends[-last:]):
        out.append([r for r in rows if a < r["s"] <= b])
    return out


def union(rs):
    tot, cur_s, cur_e = 0, None, None
    for r in sorted(rs, key=lambda r: r["s"]):
        if cur_e is None or r["s"] > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = r["s"], r["e"]
        else:
            cur_e = max(cur_e, r["e"])
    return tot + (cur_e - cur_s if cur_e is not None else 0)


def main(d="gpurun_out/r05gtrace"):
    per = {}
    for mode in ("eager", "graph"):
        st = steps(load(f"{d}/{mode}_kernel_trace.csv.gz"))
        span = sum(s[-1]["e"] - s[0]["s"] for s in st) / len(st) / 1e6
        ksum = sum(r["e"] - r["s"] for s in st for r in s) / len(st) / 1e6
        busy = sum(union(s) for s in st) / len(st) / 1e6
        qs = collections.Counter(r["q"] for s in st for r in s)
        print(f"{mode}: {len(st[0])} kernels/step, span {span:.2f} ms, kernel sum {ksum:.2f} ms, "
              f"busy union {busy:.2f} ms, queues {dict(qs)}")
        g = collections.defaultdict(float)
        for s in st:
            for r in s:
                g[r["n"]] += (r["e"] - r["s"]) / len(st) / 1e6
        per[mode] = g
    diffs = sorted(((per["graph"].get(k, 0) - per["eager"].get(k, 0), k) for k in set(per["eager"]) | set(per["graph"])),
                   reverse=True)
    print("kernel groups, graph - eager ms/step (largest first):")
    for dlt, k in diffs[:15]:
        print(f"  {dlt:+.3f}  eager {per['eager'].get(k, 0):.3f}  graph {per['graph'].get(k, 0):.3f}  {k}")
    print("  ...")
    for dlt, k in diffs[-5:]:
        print(f"  {dlt:+.3f}  eager {per['eager'].get(k, 0):.3f}  graph {per['graph'].get(k, 0):.3f}  {k}")


if __name__ == "__main__":
    main(*sys.argv[1:])
