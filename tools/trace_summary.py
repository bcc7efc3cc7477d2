"""Summarize a rocprofv3 --kernel-trace CSV: per-kernel count / mean / median (us)."""
import collections
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for r in rows:
    d[r["Kernel_Name"].split("(")[0]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k:40s} n={len(v):6d} mean={sum(v)/len(v)/1e3:9.2f}us median={statistics.median(v)/1e3:9.2f}us "
          f"total={sum(v)/1e6:9.2f}ms")
