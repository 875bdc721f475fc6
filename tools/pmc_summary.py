"""Summarise rocprofv3 counter_collection CSVs of the fvp_mlp3 kernel: median per dispatch.
usage: python tools/pmc_summary.py DIR [DIR ...]"""
import csv, glob, os, statistics, sys
for d in sys.argv[1:]:
    vals = {}
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if os.environ.get("KERNEL", "fvp_mlp3") not in r["Kernel_Name"]:
                continue
            k = (r["Counter_Name"], r["Dispatch_Id"])
            vals[k] = vals.get(k, 0.0) + float(r["Counter_Value"])
    per = {}
    for (c, _), v in vals.items():
        per.setdefault(c, []).append(v)
    print(d)
    for c in sorted(per):
        print("  %-28s %14.1f" % (c, statistics.median(per[c])))
