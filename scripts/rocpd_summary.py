"""Kernel table from a rocprofv3 SQLite output (run_results.db, the default
format without -f csv): kernels of the last `passes` passes (a pass starts at
each dispatch of `marker`), total ms per pass, share, calls per pass and
average duration -- the format of prof_summary.py.
Usage: rocpd_summary.py run_results.db [marker] [passes] [top]"""
import sqlite3
import sys

db = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "stem_fwd_kernel"
passes = int(sys.argv[3]) if len(sys.argv) > 3 else 1
top = int(sys.argv[4]) if len(sys.argv) > 4 else 40
c = sqlite3.connect(db)
rows = c.execute("select name, start, end from kernels order by start").fetchall()
starts = [s for n, s, e in rows if marker in n]
if len(starts) < passes:
    raise SystemExit(f"only {len(starts)} dispatches of {marker}")
lo = starts[-passes]
sel = [(n, s, e) for n, s, e in rows if s >= lo]
agg = {}
for n, s, e in sel:
    a = agg.setdefault(n, [0, 0])
    a[0] += e - s
    a[1] += 1
tot = sum(v[0] for v in agg.values())
for n, (t, k) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:top]:
    print(f"{t / 1e6 / passes:8.2f} ms/pass {100.0 * t / tot:6.2f}% n={k / passes:7.1f} avg={t / k / 1e3:9.1f}us "
          f"{n[:100]}")
print(f"total kernel time {tot / 1e6 / passes:.2f} ms/pass over the last {passes} passes "
      f"(window {(sel[-1][2] - lo) / 1e6 / passes:.2f} ms/pass)")
