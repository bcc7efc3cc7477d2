#!/bin/bash
# Round 3: config 1 (scaled) with the generic deferred commit (KSIM_LAZY_GEN=1)
# against the three-launch generic batches (default), interleaved on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/${TAG:-r03gen}
mkdir -p "$OUT"
for r in $(seq 1 ${REPS:-2}); do
  for v in gen nogen; do
    if [ $v == gen ]; then export KSIM_LAZY_GEN=1; else unset KSIM_LAZY_GEN; fi
    timeout -k 10 300 python3 -u bench.py --config 1 --steps 3 --warmup 1 --no-cpu > "$OUT/c1_${v}_$r.json" 2> "$OUT/c1_${v}_$r.err" || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1].split('/')[-1], '%.3f ms' % d['ms_per_step'], d['batch_stats'])" "$OUT/c1_${v}_$r.json"
  done
done
unset KSIM_LAZY_GEN
