#!/bin/bash
# Round 5 measurement set: LINES (default c1 c1a c3 c4 c4a c5 fw) as bench
# lines, each followed by the same command under rocprofv3 --kernel-trace
# --stats (kernel_stats CSV kept); TESTS=1 runs every -m gpu test and smoke()
# first.  Output under gpurun_out/${TAG}.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/${TAG:-r05final}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.txt" 2>&1 || { tail -30 "$OUT/pytest_gpu.txt"; exit 1; }
  tail -1 "$OUT/pytest_gpu.txt"
  timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.txt" 2>&1 || exit 1
  tail -1 "$OUT/smoke.txt"
fi
for c in ${LINES}; do
  case $c in
    default) args="" ;;
    c1) args="--config 1 --steps 3 --warmup 1" ;;
    c1a) args="--config 1 --mode adapt --steps 2 --warmup 1" ;;
    c3) args="--config 3 --steps 3 --warmup 1" ;;
    c4) args="--config 4 --steps 2 --warmup 1" ;;
    c4a) args="--config 4 --mode adapt --steps 2 --warmup 1" ;;
    c5) args="--config 5 --steps 1 --warmup 1" ;;
    fw) args="--mode fw" ;;
  esac
  echo "== $c: bench.py $args"
  timeout -k 10 600 python3 -u bench.py $args > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err" || { tail -5 "$OUT/bench_$c.err"; exit 1; }
  python3 - "$OUT/bench_$c.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
if "rows" in d:
    for r in d["rows"]:
        c = r.get("engine_c_driver") or {}
        print("  fw", r["nodes"], "C", round(c.get("us_per_cycle", 0), 1), "py", round(r["engine"]["us_per_cycle"], 1),
              "oracle", round(r["oracle_cpu_1thread"]["us_per_cycle"], 1))
else:
    rf = d.get("roofline", {})
    print("  %.3f ms" % d["ms_per_step"], "%.3e %s" % (d["value"], d["unit"]), d.get("batch_stats"), "vs_cpu",
          d.get("vs_cpu"), "roofline", rf.get("kernel"), rf.get("bound"), rf.get("frac"), rf.get("avg_launch_ms"))
PY
  [ "$c" = fw ] && continue
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$c" -o run --output-format csv -- \
    python3 -u bench.py $args --no-cpu > "$OUT/prof_bench_$c.json" 2> "$OUT/prof_bench_$c.err" || exit 1
  find "$OUT/prof_$c" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats_$c.csv" \;
  rm -rf "$OUT/prof_$c"
  head -4 "$OUT/kernel_stats_$c.csv" | cut -d, -f1-4 | cut -c1-120
done
