"""Effective shader clock of a kernel from one rocprofv3 pass (--pmc GRBM_GUI_ACTIVE --kernel-trace):
GRBM_GUI_ACTIVE / 8 XCDs / kernel duration, median over the kernel's dispatches (reads a few % high
below ~0.3 ms per dispatch, MI355X_MICROARCH.md 'DVFS give-back').
usage: KERNEL=substr python tools/clock_summary.py DIR"""
import csv, glob, os, statistics, sys
d = sys.argv[1]
kern = os.environ.get("KERNEL", "fvp_mlp3_kernel<1, 1, 1, 1, 5, 3")
cnt, dur = {}, {}
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"] and r["Counter_Name"] == "GRBM_GUI_ACTIVE":
            cnt[r["Dispatch_Id"]] = cnt.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"]:
            dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
ghz = [cnt[k] / 8 / dur[k] / 1e9 for k in cnt if k in dur and dur[k] > 0]
us = [dur[k] * 1e6 for k in cnt if k in dur]
print("%s: %d dispatches, duration med %.1f us, effective clock med %.3f GHz" % (
    d, len(ghz), statistics.median(us) if us else 0, statistics.median(ghz) if ghz else 0))
