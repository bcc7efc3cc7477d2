#!/bin/bash
# A/B of the batch geometry builds (csrc/Makefile variant) on one box, config 2 P100 (+ ADAPT line).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-geom}
mkdir -p "$OUT"
for v in ${VARIANTS:-base b512t8 b256t16 b512t16 base}; do
  unset KSIM_LIB_VARIANT
  [ $v != base ] && export KSIM_LIB_VARIANT=$v
  [ -n "$TILES" ] && export=1
  timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu ${BENCH_ARGS} > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.err" || exit $?
  python3 -c "
import json
d=json.loads(open('$OUT/bench_$v.json').read().strip().splitlines()[-1])
print('$v', 'value %.4e'%d['value'], 'ms/step %.3f'%d['ms_per_step'], d['batch_stats'], {k:(round(x['avg_ms']*1000,2)) for k,x in d['kernels'].items()}, 'eval %.2f us'%(d['roofline']['avg_launch_ms']*1000), 'adapt %.3e'%d.get('adapt',{}).get('value',0), d.get('adapt',{}).get('batches'))
"
done
