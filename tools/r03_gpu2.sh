#!/bin/bash
# Round 3 GPU call: framework-driven compat + race regression + batch parity
# tests, then a config-2 A/B of the FAST-key rewrite (r3base = the library of
# the previous commit), then the SQ cycle counters.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/r03b
mkdir -p "$OUT"
timeout -k 10 420 python -u -m pytest tests/test_gpu_fw.py tests/test_gpu_chain_race.py tests/test_gpu_parity.py -x -v --timeout 240 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; if [ $rc -ne 0 ]; then exit $rc; fi
for r in 1 2; do
  for v in r3base new; do
    lib=$v; [[ $v == new ]] && lib=""
    KSIM_LIB_VARIANT=$lib timeout -k 10 200 python3 -u bench.py --steps 5 --warmup 2 --no-cpu > "$OUT/c2_${v}_$r.json" 2> "$OUT/c2_${v}_$r.err" || exit $?
  done
done
python3 - "$OUT" <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/c2_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    k = d["kernels"]
    print(f.split("/")[-1], "%.3f ms" % d["ms_per_step"], "adapt %.3f ms" % d["adapt"]["ms_per_step"],
          {n: round(v["avg_ms"] * 1e3, 2) for n, v in k.items()})
PY
TAG=r03sq bash tools/r03_sq.sh
