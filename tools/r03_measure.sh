#!/bin/bash
# Round 3: parity tests (TESTS), then one bench line per config in CONFIGS
# ("1", "2", "3", "2a" = config 2 ADAPT mode, ...), JSON lines under gpurun_out/$TAG.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/${TAG:-r03m}
mkdir -p "$OUT"
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -v --timeout 240 --timeout-method thread > "$OUT/pytest.log" 2>&1
  rc=$?; tail -3 "$OUT/pytest.log"; if [ $rc -ne 0 ]; then exit $rc; fi
fi
for cfg in ${CONFIGS:-2}; do
  mode=p100; c=$cfg
  if [[ $cfg == *a ]]; then mode=adapt; c=${cfg%a}; fi
  timeout -k 10 400 python3 -u bench.py --config $c --mode $mode --steps ${STEPS:-3} --warmup 1 ${BENCH_ARGS} \
    > "$OUT/bench_c$cfg.json" 2> "$OUT/bench_c$cfg.err" || exit $?
  python3 - "$OUT/bench_c$cfg.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = {n: round(v["avg_ms"] * 1e3, 2) for n, v in d["kernels"].items() if not n.startswith("_")}
cb = d.get("cpu_baseline", {})
print(sys.argv[1].split("/")[-1], "%.3f ms" % d["ms_per_step"], "%.3e evals/s" % d["value"], d["batch_stats"], k,
      "cpu %.3e x%s" % (cb.get("value", 0), cb.get("cores")), "vs_cpu %.1f" % d.get("vs_cpu", 0))
PY
done
