#!/bin/bash
# Round 3: deferred commit on both batch paths -- the whole GPU suite, then
# config 2 (P100 line + ADAPT line) and config 4 ADAPT, default against
# KSIM_NO_LAZY=1, same box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/${TAG:-r03lazy2}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest ${TESTS:-tests -m gpu} -x -v --timeout 240 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; if [ $rc -ne 0 ]; then exit $rc; fi
for r in 1 2; do
  for v in lazy nolazy; do
    if [ $v == nolazy ]; then export KSIM_NO_LAZY=1; else unset KSIM_NO_LAZY; fi
    timeout -k 10 200 python3 -u bench.py --steps 5 --warmup 2 --no-cpu > "$OUT/c2_${v}_$r.json" 2> "$OUT/c2_${v}_$r.err" || exit $?
  done
done
for v in lazy nolazy; do
  if [ $v == nolazy ]; then export KSIM_NO_LAZY=1; else unset KSIM_NO_LAZY; fi
  timeout -k 10 300 python3 -u bench.py --config 4 --mode adapt --steps 2 --warmup 1 --no-cpu > "$OUT/c4a_${v}.json" 2> "$OUT/c4a_${v}.err" || exit $?
done
unset KSIM_NO_LAZY
python3 - "$OUT" <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/c*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    k = d["kernels"]
    print(f.split("/")[-1], "%.3f ms" % d["ms_per_step"], "%.3e" % d["value"], "adapt %s" % (d.get("adapt") or {}).get("ms_per_step"), d["batch_stats"],
          {n: round(v["avg_ms"] * 1e3, 2) for n, v in k.items() if not n.startswith("_")})
PY
