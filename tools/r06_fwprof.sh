#!/bin/bash
# Round 6: the drop-in delta tests, then bench.py --mode fw plain and under
# rocprofv3 --kernel-trace --stats.  Output under gpurun_out/${TAG:-r06fw}.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/${TAG:-r06fw}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "${K:-snapshot}" \
  > "$OUT/pytest_gpu.txt" 2>&1 || { tail -30 "$OUT/pytest_gpu.txt"; exit 1; }
tail -2 "$OUT/pytest_gpu.txt"
timeout -k 10 500 python3 -u bench.py --mode fw > "$OUT/bench_fw.json" 2> "$OUT/bench_fw.err" || { tail -5 "$OUT/bench_fw.err"; exit 1; }
python3 - "$OUT/bench_fw.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", round(d["value"], 1), d["unit"])
for r in d["rows"]:
    out = {"nodes": r["nodes"]}
    for k in ("engine", "engine_c_driver", "engine_c_driver_deltas", "oracle_cpu_1thread"):
        if r.get(k):
            out[k] = round(r[k]["us_per_cycle"], 1)
    print(out)
    dd = r.get("engine_c_driver_deltas")
    if dd:
        print("  split", {k: round(v, 1) for k, v in dd["us_per_call"].items()}, dd["events"])
PY
if [ -n "$PROF" ]; then
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o fw -- python3 bench.py --mode fw > "$OUT/bench_fw_prof.json" 2> "$OUT/bench_fw_prof.err" || exit $?
  python3 tools/kstats.py $(find "$OUT/prof" -name '*results.db' | head -1) | head -30
  find "$OUT/prof" -name '*kernel_stats.csv' | head -1 | xargs -r head -30
fi
