"""Exchange-kernel duration statistics from a rocprofv3 kernel trace of tools/peer_floor.py.
usage: python tools/peer_floor_stats.py LABEL TRACE_DIR   (finds *kernel_trace.csv under TRACE_DIR)
The rank that reaches an exchange second waits for nothing, so the lower half of the distribution is
the exchange itself; prints min / p10 / p25 / median of the lower half / median, in us."""
import csv
import glob
import os
import sys

import numpy as np

label, d = sys.argv[1], sys.argv[2]
files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
if not files:
    sys.exit("no kernel_trace.csv under %s" % d)
us = []
with open(files[0]) as f:
    for row in csv.DictReader(f):
        if "peer_" in row["Kernel_Name"]:
            us.append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)
us = np.sort(np.array(us))
if us.size == 0:
    sys.exit("no peer exchange kernels in %s" % files[0])
lower = us[: us.size // 2]
print("%-8s exchanges %d  min %.2f  p10 %.2f  p25 %.2f  median of lower half %.2f  median %.2f" % (
    label, us.size, us[0], np.percentile(us, 10), np.percentile(us, 25), np.median(lower), np.median(us)))
