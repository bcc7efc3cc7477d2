#!/bin/bash
# GPU parity tests named by K, then bench.py $ARGS (default: config 4 P100) on the
# default library and on KSIM_LIB_VARIANT=$1, alternating; output gpurun_out/$2
set -o pipefail
ARGS=${ARGS:---config 4 --steps 2 --warmup 1}
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/$2; mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" \
    > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
  tail -2 $OUT/pytest.txt
fi
for r in 1 2; do
  timeout -k 10 400 python3 -u bench.py $ARGS --no-cpu > $OUT/cur_$r.json 2>$OUT/cur_$r.err || exit 1
  KSIM_LIB_VARIANT=$1 timeout -k 10 400 python3 -u bench.py $ARGS --no-cpu > $OUT/$1_$r.json 2>$OUT/$1_$r.err || exit 1
done
python3 - $OUT <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], round(d["ms_per_step"], 2), d.get("batch_stats"), d["roofline"].get("live_avg_launch_ms"))
PY
