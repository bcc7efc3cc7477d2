#!/bin/bash
# Round 6 same-box A/B: the default library against KSIM_LIB_VARIANT flavors
# ($VARIANTS), alternating, $REPS rounds of bench.py $ARGS (default: config 2).
# Output under gpurun_out/${TAG}.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/${TAG:-r06ab}
mkdir -p "$OUT"
ARGS=${ARGS:---no-cpu}
for r in $(seq 1 ${REPS:-2}); do
  timeout -k 10 300 python3 -u bench.py $ARGS > $OUT/cur_$r.json 2>$OUT/cur_$r.err || { tail -5 $OUT/cur_$r.err; exit 1; }
  for v in $VARIANTS; do
    KSIM_LIB_VARIANT=$v timeout -k 10 300 python3 -u bench.py $ARGS > $OUT/${v}_$r.json 2>$OUT/${v}_$r.err || { tail -5 $OUT/${v}_$r.err; exit 1; }
  done
done
python3 - $OUT <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    r = d.get("roofline", {})
    print(f.split("/")[-1], round(d["ms_per_step"], 3), r.get("live_avg_launch_ms"), d.get("batch_stats", {}).get("batches") if isinstance(d.get("batch_stats"), dict) else d.get("batch_stats"))
PY
