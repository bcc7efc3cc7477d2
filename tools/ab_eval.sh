#!/bin/bash
# A/B of the batch evaluation form on one box: k_batch_top (default) vs the
# round-1 per-tile lists + k_batch_merge (KSIM_BATCH_TILES=1); config 2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-ab}
mkdir -p "$OUT"
for v in ${VARIANTS:-top tiles top}; do
  unset KSIM_BATCH_TILES KSIM_TOP_THREADS
  case $v in tiles) export KSIM_BATCH_TILES=1 ;; top512) export KSIM_TOP_THREADS=512 ;; esac
  timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu ${BENCH_ARGS} > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.err" || exit $?
  python3 -c "
import json,sys
d=json.loads(open('$OUT/bench_$v.json').read().strip().splitlines()[-1])
print('$v', 'value %.4e'%d['value'], 'ms/step %.3f'%d['ms_per_step'], {k:(round(x['avg_ms']*1000,2),x['launches']) for k,x in d['kernels'].items()}, 'eval %.2f us'%(d['roofline']['avg_launch_ms']*1000), 'adapt', d.get('adapt',{}).get('value'))
"
done
