"""Per-kernel average duration table from a rocprofv3 results .db (kernel-trace run).
usage: python tools/ktime.py path/to/results.db [name-filter]"""
import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
flt = sys.argv[2] if len(sys.argv) > 2 else ""
for name, calls, tot, avg, pct in c.execute("select * from top_kernels"):
    if flt in name:
        print("%-60s calls %5d  avg %9.2f us  total %10.1f us  %5.1f%%" % (name[:60], calls, avg, tot, pct))
