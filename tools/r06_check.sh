#!/bin/bash
# Round 6 check on one box: every -m gpu test (one process), smoke, the
# default bench line, then BENCH_CONFIGS lines (bench.py --config ...).
# Output under gpurun_out/${TAG:-r06check}.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/${TAG:-r06check}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${K:+-k "$K"} \
    > "$OUT/pytest_gpu.txt" 2>&1 || { tail -30 "$OUT/pytest_gpu.txt"; exit 1; }
  tail -3 "$OUT/pytest_gpu.txt"
fi
[ -n "$NOSMOKE" ] || {
  timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.txt" 2>&1 || exit $?
  tail -1 "$OUT/smoke.txt"
}
[ -n "$NODEFAULT" ] || {
  timeout -k 10 400 python3 -u bench.py ${BENCH_ARGS} > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || exit $?
  tail -c 400 "$OUT/bench_default.json"; echo
}
for c in ${BENCH_CONFIGS}; do
  case $c in
    1) args="--config 1 --steps 3 --warmup 1" ;;
    1a) args="--config 1 --mode adapt --steps 2 --warmup 1" ;;
    3) args="--config 3 --steps 3 --warmup 1" ;;
    4) args="--config 4 --steps 2 --warmup 1" ;;
    4a) args="--config 4 --mode adapt --steps 2 --warmup 1" ;;
    5) args="--config 5 --steps 1 --warmup 1" ;;
    2a) args="--mode adapt --no-adapt --steps 5 --warmup 2" ;;
    fw) args="--mode fw" ;;
  esac
  timeout -k 10 500 python3 -u bench.py $args > "$OUT/bench_config$c.json" 2> "$OUT/bench_config$c.err" || exit $?
  python3 - "$OUT/bench_config$c.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
if "rows" in d:
    for r in d["rows"]:
        out = {"nodes": r["nodes"]}
        for k in ("engine", "engine_c_driver", "engine_c_driver_deltas", "oracle_cpu_1thread"):
            if r.get(k):
                out[k] = round(r[k]["us_per_cycle"], 1)
        if r.get("engine_c_driver_deltas"):
            out["split"] = {k: round(v, 1) for k, v in r["engine_c_driver_deltas"]["us_per_call"].items()}
            out["events"] = r["engine_c_driver_deltas"]["events"]
        print(sys.argv[1].split("/")[-1], out)
else:
    print(sys.argv[1].split("/")[-1], "%.3f ms" % d["ms_per_step"], "%.3e evals/s" % d["value"], d.get("batch_stats"),
          "vs_cpu %s" % d.get("vs_cpu"), "host_compile %s" % {k: v for k, v in (d.get("host_compile") or {}).items()
                                                                if k.endswith("_s")})
PY
done
