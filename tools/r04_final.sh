#!/bin/bash
# Round 4 closing set on one box: smoke, the default bench line (config 2,
# with CPU baseline), its rocprof kernel stats, and one line per other config
# (1 scaled, 3, 4 ADAPT, 5, 2 ADAPT).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/${TAG:-r04final}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.txt" 2>&1 || { tail -30 "$OUT/pytest_gpu.txt"; exit 1; }
  tail -2 "$OUT/pytest_gpu.txt"
fi
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.txt" 2>&1 || exit $?
timeout -k 10 400 python3 -u bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || exit $?
tail -c 300 "$OUT/bench_default.json"; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv -- \
  python3 -u bench.py --no-cpu > "$OUT/bench_rocprof.json" 2> "$OUT/bench_rocprof.err" || exit $?
find "$OUT/stats" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats_config2.csv" \;
for c in ${CONFIGS:-1 1a 3 4a 5 2a fw}; do
  case $c in
    1) args="--config 1 --steps 3 --warmup 1" ;;
    1a) args="--config 1 --mode adapt --steps 2 --warmup 1" ;;
    3) args="--config 3 --steps 3 --warmup 1" ;;
    4a) args="--config 4 --mode adapt --steps 2 --warmup 1" ;;
    5) args="--config 5 --steps 1 --warmup 1" ;;
    2a) args="--mode adapt --no-adapt --steps 5 --warmup 2" ;;
    fw) args="--mode fw" ;;
  esac
  timeout -k 10 500 python3 -u bench.py $args > "$OUT/bench_config$c.json" 2> "$OUT/bench_config$c.err" || exit $?
  python3 - "$OUT/bench_config$c.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
cb = d.get("cpu_baseline") or {}
if "rows" in d:
    print(sys.argv[1].split("/")[-1], [(r["nodes"], round(r["engine"]["us_per_cycle"], 1),
                                       round(r["oracle_cpu_1thread"]["us_per_cycle"], 1)) for r in d["rows"]])
else:
    print(sys.argv[1].split("/")[-1], "%.3f ms" % d["ms_per_step"], "%.3e evals/s" % d["value"], d["batch_stats"],
          "vs_cpu %s" % d.get("vs_cpu"))
PY
done
