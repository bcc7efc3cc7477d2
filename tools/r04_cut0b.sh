#!/bin/bash
# k_adapt_cut0 on every ADAPT window path: the ADAPT / shard GPU tests, then
# config 4 ADAPT (lazy) and config 2 ADAPT lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/${TAG:-r04cut0b}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_round2.py tests/test_gpu_shard.py -m gpu -x -v \
  --timeout 200 --timeout-method thread > "$OUT/pytest.txt" 2>&1 || { tail -30 "$OUT/pytest.txt"; exit 1; }
tail -2 "$OUT/pytest.txt"
for c in 4a 2a; do
  case $c in
    4a) args="--config 4 --mode adapt --steps 2 --warmup 1 --no-cpu" ;;
    2a) args="--mode adapt --no-adapt --steps 5 --warmup 2 --no-cpu" ;;
  esac
  timeout -k 10 400 python3 -u bench.py $args > "$OUT/bench_config$c.json" 2> "$OUT/bench_config$c.err" || exit $?
  python3 - "$OUT/bench_config$c.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split("/")[-1], "%.3f ms" % d["ms_per_step"], "%.3e" % d["value"],
      {k: round(v["avg_ms"] * 1e3, 2) for k, v in d["kernels"].items() if "avg_ms" in v})
PY
done
