#!/bin/bash
# ADAPT first-round cuts (k_adapt_cut0): the ADAPT parity tests, then config 4 ADAPT.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/${TAG:-r04gc}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_round2.py -m gpu -x -v -k "adapt" \
  --timeout 200 --timeout-method thread > "$OUT/pytest_adapt.txt" 2>&1 || { tail -30 "$OUT/pytest_adapt.txt"; exit 1; }
tail -2 "$OUT/pytest_adapt.txt"
timeout -k 10 400 python3 -u bench.py --config 4 --mode adapt --steps 2 --warmup 1 --no-cpu \
  > "$OUT/bench_config4a.json" 2> "$OUT/bench_config4a.err" || exit $?
python3 - "$OUT/bench_config4a.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("%.3f ms" % d["ms_per_step"], "%.3e" % d["value"], {k: round(v["avg_ms"] * 1e3, 2) for k, v in d["kernels"].items() if "avg_ms" in v})
PY
