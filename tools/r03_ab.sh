#!/bin/bash
# Round 3 A/B: parity tests on the default library (TESTS), then config 2 for
# every library variant in VARIANTS ("" = default; a tag loads
# libksim_engine_<tag>.so), interleaved, REPS rounds; a summary line per run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/${TAG:-r03ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -v --timeout 240 --timeout-method thread > "$OUT/pytest.log" 2>&1
  rc=$?; tail -3 "$OUT/pytest.log"; if [ $rc -ne 0 ]; then exit $rc; fi
fi
for r in $(seq 1 ${REPS:-2}); do
  for v in ${VARIANTS:-default}; do
    lib=$v; [[ $v == default ]] && lib=""
    KSIM_LIB_VARIANT=$lib timeout -k 10 200 python3 -u bench.py --steps 5 --warmup 2 --no-cpu ${BENCH_ARGS} > "$OUT/c_${v}_$r.json" 2> "$OUT/c_${v}_$r.err" || exit $?
  done
done
python3 - "$OUT" <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/c_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    k = d["kernels"]
    ad = d.get("adapt", {}).get("ms_per_step", 0)
    print(f.split("/")[-1], "%.3f ms" % d["ms_per_step"], "adapt %.3f ms" % ad, d["batch_stats"],
          {n: round(v["avg_ms"] * 1e3, 2) for n, v in k.items() if not n.startswith("_")})
PY
