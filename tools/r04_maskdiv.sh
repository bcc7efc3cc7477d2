#!/bin/bash
# A/B of the ADAPT mask grid (pods per block = node blocks / KSIM_MASK_DIV):
# config 2 ADAPT and config 4 ADAPT per build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/${TAG:-r04maskdiv}
mkdir -p "$OUT"
for v in "" div4 div2 div1; do
  for c in 2a 4a; do
    case $c in
      4a) args="--config 4 --mode adapt --steps 2 --warmup 1 --no-cpu" ;;
      2a) args="--mode adapt --no-adapt --steps 5 --warmup 2 --no-cpu" ;;
    esac
    KSIM_LIB_VARIANT=$v timeout -k 10 300 python3 -u bench.py $args > "$OUT/bench_${v:-div8}_$c.json" 2> "$OUT/bench_${v:-div8}_$c.err" || exit $?
    python3 - "$OUT/bench_${v:-div8}_$c.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split("/")[-1], "%.3f ms" % d["ms_per_step"],
      {k: round(v["avg_ms"] * 1e3, 2) for k, v in d["kernels"].items() if "avg_ms" in v})
PY
  done
done
