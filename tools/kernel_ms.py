"""profiles/kernel_ms.json: in-graph mean durations of the bench lines'
dominant kernels from committed rocprofv3 summaries (bench.py prices a line's
roofline at this figure when its live back-to-back time differs by > 5 %).
Usage: python tools/kernel_ms.py <config> <mode> <nodes> <kernel> <summary> [...]
  summary: a rocprofv3 results .db or a *kernel_stats.csv under profiles/."""
import csv
import json
import os
import sqlite3
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "profiles", "kernel_ms.json")
# bench kernel-table slot -> the kernel symbol rocprofv3 reports
SYMBOL = {"k_adapt_mask": "k_adapt_mask_ns"}


def mean_ms(path, kernel):
    """Mean duration (ms) of the kernel whose name starts with ksim::<kernel>< or ( (template instances
    summed by count)."""
    sym = SYMBOL.get(kernel, kernel)
    keys = (f"ksim::{sym}<", f"ksim::{sym}(")
    n = tot = 0
    if path.endswith(".db"):
        for name, cnt, s in sqlite3.connect(path).execute(
                "select name, count(*), sum(end - start) from kernels group by name"):
            if any(k in name for k in keys):
                n, tot = n + cnt, tot + s * 1e-6
    else:
        for row in csv.DictReader(open(path)):
            if any(k in row["Name"] for k in keys):
                c = int(row["Calls"])
                n, tot = n + c, tot + float(row["TotalDurationNs"]) * 1e-6
    return tot / n if n else None, n


def main():
    a = sys.argv[1:]
    entries = json.load(open(OUT)) if os.path.exists(OUT) else []
    for i in range(0, len(a), 5):
        cfg, mode, nodes, kernel, path = int(a[i]), a[i + 1], int(a[i + 2]), a[i + 3], a[i + 4]
        ms, n = mean_ms(path, kernel)
        if ms is None:
            raise SystemExit(f"{kernel} not in {path}")
        entries = [e for e in entries if not (e["config"] == cfg and e["mode"] == mode and e["nodes"] == nodes
                                              and e["kernel"] == kernel)]
        entries.append({"config": cfg, "mode": mode, "nodes": nodes, "kernel": kernel, "avg_ms": ms,
                        "launches": n, "source": os.path.relpath(path, ROOT)})
        print(entries[-1])
    json.dump(entries, open(OUT, "w"), indent=1)


if __name__ == "__main__":
    main()
