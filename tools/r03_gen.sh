#!/bin/bash
# Round 3: config 1 (scaled), interleaved on one box: the static-class FAST
# keys (default), the same with the deferred commit (KSIM_LAZY_STAB=1), and
# the generic keys (KSIM_NO_STAB=1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/${TAG:-r03gen}
mkdir -p "$OUT"
for r in $(seq 1 ${REPS:-2}); do
  for v in ${GVARIANTS:-stab stablazy nostab}; do
    unset KSIM_NO_STAB KSIM_LAZY_GEN KSIM_NO_LAZY KSIM_LAZY_STAB
    [ $v == nostab ] && export KSIM_NO_STAB=1
    [ $v == stablazy ] && export KSIM_LAZY_STAB=1
    [ $v == lazygen ] && export KSIM_NO_STAB=1 KSIM_LAZY_GEN=1
    timeout -k 10 300 python3 -u bench.py --config 1 --steps 3 --warmup 1 --no-cpu > "$OUT/c1_${v}_$r.json" 2> "$OUT/c1_${v}_$r.err" || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1].split('/')[-1], '%.3f ms' % d['ms_per_step'], d['batch_stats'], {n: round(v['avg_ms'] * 1e3, 2) for n, v in d['kernels'].items() if not n.startswith('_')})" "$OUT/c1_${v}_$r.json"
  done
done
unset KSIM_NO_STAB KSIM_LAZY_GEN KSIM_NO_LAZY KSIM_LAZY_STAB
