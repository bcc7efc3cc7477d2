#!/bin/bash
# A/B: default library vs KSIM_LIB_VARIANT=$1, alternating, config 2 bench lines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/$2; mkdir -p $OUT
for r in 1 2; do
  timeout -k 10 300 python3 -u bench.py --no-cpu > $OUT/cur_$r.json 2>$OUT/cur_$r.err || exit 1
  KSIM_LIB_VARIANT=$1 timeout -k 10 300 python3 -u bench.py --no-cpu > $OUT/$1_$r.json 2>$OUT/$1_$r.err || exit 1
done
python3 - $OUT $1 <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], round(d["ms_per_step"], 3), d["roofline"].get("live_avg_launch_ms"))
PY
