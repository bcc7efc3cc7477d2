#!/bin/bash
# Round 5: the drop-in cycle (bench.py --mode fw: Python loop and C driver),
# then the same under rocprofv3 kernel trace.  Output under gpurun_out/${TAG}.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/${TAG:-r05fw}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py --mode fw > "$OUT/bench_fw.json" 2> "$OUT/bench_fw.err" || { tail -5 "$OUT/bench_fw.err"; exit 1; }
python3 - "$OUT/bench_fw.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for r in d["rows"]:
    c = r.get("engine_c_driver") or {}
    print(r["nodes"], "py", round(r["engine"]["us_per_cycle"], 1), "C", round(c.get("us_per_cycle", 0), 1),
          {k: round(v, 1) for k, v in c.get("us_per_call", {}).items()}, c.get("answered"),
          "oracle", round(r["oracle_cpu_1thread"]["us_per_cycle"], 1))
PY
if [ -n "$PROF" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o fw -- python3 bench.py --mode fw > "$OUT/bench_fw_prof.json" 2> "$OUT/bench_fw_prof.err" || exit $?
  python3 tools/kstats.py $(find "$OUT/prof" -name '*results.db' | head -1) | head -12
fi
