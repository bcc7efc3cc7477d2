"""Per-kernel mean per dispatch of every counter under a rocprofv3 --pmc output
tree (counters summed over the XCD / SE instances of one dispatch)."""
import collections
import csv
import glob
import os
import statistics
import sys

per = collections.defaultdict(float)
for f in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").replace("ksim::", "")
        d = r.get("Dispatch_Id") or r.get("Correlation_Id")
        per[(k, r["Counter_Name"], f, d)] += float(r["Counter_Value"])
acc = collections.defaultdict(list)
for (k, c, _, _), v in per.items():
    acc[(k, c)].append(v)
for (k, c), v in sorted(acc.items()):
    print(f"{k:28s} {c:22s} n={len(v):5d} mean={statistics.mean(v):16.1f}")
