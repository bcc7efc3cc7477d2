#!/bin/bash
# Config-2 A/B on one box: the default library against KSIM_LIB_VARIANT
# flavors (args), REPS rounds interleaved; optional parity tests first (TESTS).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/${TAG:-r03ab}
mkdir -p "$OUT"
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -v --timeout 240 --timeout-method thread > "$OUT/pytest.log" 2>&1
  rc=$?; tail -3 "$OUT/pytest.log"; if [ $rc -ne 0 ]; then exit $rc; fi
fi
for r in $(seq 1 ${REPS:-2}); do
  for v in new "$@"; do
    lib=$v; envset=""; [[ $v == new ]] && lib=""
    # env_NAME=VALUE: the default library with an environment switch (A/B switches read at run time)
    if [[ $v == env_* ]]; then lib=""; envset=${v#env_}; fi
    env $envset KSIM_LIB_VARIANT=$lib timeout -k 10 200 python3 -u bench.py --steps 5 --warmup 2 --no-cpu ${BENCH_ARGS} > "$OUT/c2_${v}_$r.json" 2> "$OUT/c2_${v}_$r.err" || exit $?
  done
done
python3 - "$OUT" <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/c2_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    k = d["kernels"]
    a = d.get("adapt", {}).get("ms_per_step", 0)
    print(f.split("/")[-1], "%.3f ms" % d["ms_per_step"], "adapt %.3f ms" % a,
          {n: round(v["avg_ms_events"] * 1e3, 2) for n, v in k.items() if not n.startswith("_")})
PY
