"""Per-kernel count / mean / total from a rocprofv3 results database.
Usage: python tools/kstats.py gpurun_out/<tag>/prof/<tag>_results.db"""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
rows = db.execute("select name, count(*), avg(end-start), sum(end-start) from kernels group by name "
                  "order by sum(end-start) desc").fetchall()
for name, n, avg, tot in rows:
    print(f"{name[:90]:90s} {n:7d} {avg / 1e3:9.2f} us {tot / 1e6:9.2f} ms")
