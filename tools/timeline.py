"""Kernel timeline of the last CG solve in a rocprofv3 kernel-trace .db: start offset, duration and
the gap before each kernel.  usage: python tools/timeline.py results.db [kernels_per_solve]"""
import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
k = int(sys.argv[2]) if len(sys.argv) > 2 else 12
tabs = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
kt = [t for t in tabs if t.lower().startswith("rocpd_kernel_dispatch") or t == "kernels"]
t = "kernels" if "kernels" in tabs else kt[0]
cols = [r[1] for r in c.execute("pragma table_info(%s)" % t)]
name_col = "name" if "name" in cols else ("kernel_name" if "kernel_name" in cols else None)
rows = list(c.execute("select %s, start, end from %s order by start" % (name_col, t)))
rows = rows[-k:]
t0 = rows[0][1]
prev = None
for name, s, e in rows:
    gap = (s - prev) / 1e3 if prev is not None else 0.0
    print("%8.2f us  dur %6.2f  gap %6.2f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, gap, name[:70]))
    prev = e
print("span %.2f us" % ((rows[-1][2] - t0) / 1e3))
