"""Per-launch HBM traffic of the FVP kernel from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE),
corrected per MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE reports half the bytes of wide
(16 B/lane) coalesced streaming reads -> doubled; WRITE_SIZE is exact for 16-B streaming stores.
Counters are in KiB.  usage: python tools/pmc_traffic.py FETCH_CSV WRITE_CSV OUT_JSON"""
import csv, json, os, statistics, sys

KERNEL = os.environ.get("KERNEL", "fvp_mlp3_kernel<1, 1, 1, 1, 5, 2>")   # MODE 2: the cached-forward FVP


def per_dispatch(path, counter):
    vals = {}
    for r in csv.DictReader(open(path)):
        if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return list(vals.values())


f = per_dispatch(sys.argv[1], "FETCH_SIZE")
w = per_dispatch(sys.argv[2], "WRITE_SIZE")
fetch = 2.0 * statistics.median(f) * 1024
write = statistics.median(w) * 1024
out = {"kernel": KERNEL + " " + os.environ.get("LABEL", "(plain FVP, cached forward)"), "workload": os.environ.get("WORKLOAD", "armDOF_0 N=50000"),
       "fetch_bytes": fetch, "write_bytes": write, "traffic_bytes": fetch + write,
       "raw_FETCH_SIZE_KiB": statistics.median(f), "raw_WRITE_SIZE_KiB": statistics.median(w),
       "dispatches": [len(f), len(w)], "correction": "FETCH_SIZE x2 (gfx950 wide-read undercount)"}
json.dump(out, open(sys.argv[3], "w"), indent=1)
print(json.dumps(out))
