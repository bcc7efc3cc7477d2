"""Summarise rocprofv3 --pmc CSVs (tools/pmc_traffic.sh) into per-launch HBM bytes.

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE is in KiB and reports
half the bytes of a coalesced streaming read, so reads = 2 x FETCH_SIZE x 1024;
WRITE_SIZE x 1024 is exact for streaming stores.
"""
import csv
import glob
import json
import os
import statistics
import sys

out = sys.argv[1]
vals = {}
for f in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        name = r.get("Counter_Name")
        v = float(r.get("Counter_Value", "nan"))
        k = r.get("Kernel_Name", "").split("(")[0]
        key = (k, name)
        vals.setdefault(key, {})
        d = r.get("Dispatch_Id") or r.get("Correlation_Id") or str(len(vals[key]))
        vals[key][d] = vals[key].get(d, 0.0) + v     # sum over XCD/SE instances of one dispatch
res = {}
for (k, name), per in vals.items():
    xs = list(per.values())
    res.setdefault(k, {})[name] = {"dispatches": len(xs), "mean": statistics.mean(xs),
                                   "median": statistics.median(xs)}
for k, d in res.items():
    fetch = d.get("FETCH_SIZE", {}).get("mean")
    write = d.get("WRITE_SIZE", {}).get("mean")
    if fetch is not None:
        d["hbm_read_bytes_per_launch"] = 2 * fetch * 1024
    if write is not None:
        d["hbm_write_bytes_per_launch"] = write * 1024
    if fetch is not None and write is not None:
        d["hbm_bytes_per_launch"] = 2 * fetch * 1024 + write * 1024
    h, m = d.get("TCC_HIT_sum", {}).get("mean"), d.get("TCC_MISS_sum", {}).get("mean")
    if h is not None and m is not None and h + m > 0:
        d["l2_hit_rate"] = h / (h + m)
print(json.dumps(res, indent=1))
