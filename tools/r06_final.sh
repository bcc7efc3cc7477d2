#!/bin/bash
# Round 6 closing set on one box: every -m gpu test (one process), smoke, the
# default bench line and the secondary lines (bench.py JSON with the CPU
# baseline), then rocprofv3 kernel stats of each line (no CPU baseline).
# Output under gpurun_out/${TAG:-r06final}; each GPU step under its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/${TAG:-r06final}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.txt" 2>&1 || { tail -30 "$OUT/pytest_gpu.txt"; exit 1; }
  tail -1 "$OUT/pytest_gpu.txt"
  timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.txt" 2>&1 || exit $?
  tail -1 "$OUT/smoke.txt"
fi
line() {  # label bench-args
  local label=$1; shift
  timeout -k 10 600 python3 -u bench.py "$@" > "$OUT/bench_$label.json" 2> "$OUT/bench_$label.err" || { tail -5 "$OUT/bench_$label.err"; exit 1; }
  python3 - "$OUT/bench_$label.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
if "rows" in d:
    print(sys.argv[1].split("/")[-1], [(r["nodes"], round(r.get("engine_c_driver_deltas", r.get("engine_c_driver", {})).get("us_per_cycle", 0), 1)) for r in d["rows"]])
else:
    print(sys.argv[1].split("/")[-1], "%.3f ms" % d["ms_per_step"], "%.3e evals/s" % d["value"], d.get("batch_stats"), "vs_cpu %.1f" % (d.get("vs_cpu") or 0))
PY
}
prof() {  # label bench-args
  local label=$1; shift
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o "$label" --output-format csv -- \
    python3 bench.py --no-cpu "$@" > "$OUT/prof_$label.json" 2> "$OUT/prof_$label.err" || { tail -5 "$OUT/prof_$label.err"; exit 1; }
  cp "$OUT/prof/${label}_kernel_stats.csv" "$OUT/kernel_stats_$label.csv" 2>/dev/null
  rm -f "$OUT/prof/${label}_kernel_trace.csv" "$OUT/prof/${label}_results.db"
}
for l in ${LINES:-default c3 c1 c1a c2a c4 c4a c5 fw}; do
  case $l in
    default) args="" ;;
    c1) args="--config 1 --steps 3 --warmup 1" ;;
    c1a) args="--config 1 --mode adapt --steps 2 --warmup 1" ;;
    c2a) args="--mode adapt --no-adapt --steps 5 --warmup 2" ;;
    c3) args="--config 3 --steps 3 --warmup 1" ;;
    c4) args="--config 4 --steps 2 --warmup 1" ;;
    c4a) args="--config 4 --mode adapt --steps 2 --warmup 1" ;;
    c5) args="--config 5 --steps 1 --warmup 1" ;;
    fw) args="--mode fw" ;;
  esac
  line $l $args || exit 1
  [ "$l" = fw ] || [ -n "$NOPROF" ] || prof $l $args || exit 1
done
echo done
