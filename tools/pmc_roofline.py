"""Summarise tools/pmc_roofline.sh: per-launch HBM bytes and instruction counts.

gfx950 corrections (MI355X_MICROARCH.md HBM section): FETCH_SIZE is in KiB and
reports half the bytes of a coalesced streaming read (reads = 2 x FETCH_SIZE x
1024); WRITE_SIZE x 1024 is exact for streaming stores.  SQ counters are summed
over the XCD / SE instances of one dispatch, then averaged over dispatches.
Output: {label: {kernel, counters..., hbm_bytes_per_launch, valu_insts_per_launch, ...}}.
"""
import csv
import glob
import json
import os
import statistics
import sys

SIZES = {"config2": (5000, 256), "config3": (10000, 1)}   # nodes, pods per launch

out = sys.argv[1]
res = {}
for label_dir in sorted(glob.glob(os.path.join(out, "*"))):
    if not os.path.isdir(label_dir):
        continue
    label = os.path.basename(label_dir)
    per = {}
    kernel = None
    for f in glob.glob(os.path.join(label_dir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            kernel = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").replace("ksim::", "")
            d = r.get("Dispatch_Id") or r.get("Correlation_Id")
            key = (r["Counter_Name"], d)
            per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
    means = {}
    for (name, _), v in per.items():
        means.setdefault(name, []).append(v)
    c = {k: statistics.mean(v) for k, v in means.items()}
    nodes, pods = SIZES.get(label, (None, None))
    e = {"kernel": kernel, "nodes": nodes, "pods_per_launch": pods,
         "dispatches": {k: len(v) for k, v in means.items()}, "counters_mean_per_launch": c}
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        e["hbm_read_bytes_per_launch"] = 2 * c["FETCH_SIZE"] * 1024
        e["hbm_write_bytes_per_launch"] = c["WRITE_SIZE"] * 1024
        e["hbm_bytes_per_launch"] = e["hbm_read_bytes_per_launch"] + e["hbm_write_bytes_per_launch"]
    if "SQ_INSTS_VALU" in c:
        e["valu_insts_per_launch"] = c["SQ_INSTS_VALU"]
        e["salu_insts_per_launch"] = c.get("SQ_INSTS_SALU")
        if nodes and pods:
            e["valu_insts_per_eval_lane"] = c["SQ_INSTS_VALU"] * 64 / (nodes * pods)
    res[label] = e
print(json.dumps(res, indent=1))
