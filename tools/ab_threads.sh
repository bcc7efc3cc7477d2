#!/bin/bash
# A/B of k_batch_top's threads per pod (KSIM_TOP_THREADS) on config 2 and config 4 (1 GPU).
set -o pipefail
mkdir -p gpurun_out
for t in 1024 512 256; do
  KSIM_TOP_THREADS=$t timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/abt_$t.json 2> gpurun_out/abt_$t.err || exit $?
  python3 -c "
import json;d=json.load(open('gpurun_out/abt_$t.json'));r=d['roofline']
print('threads $t', round(d['ms_per_step'],3), 'ms', '%.3e'%d['value'], d['batch_stats'], 'eval us', round(r['avg_launch_ms']*1e3,2), 'valu', r.get('valu') and round(r['valu']['frac'],3), 'adapt', '%.3e'%d['adapt']['value'])"
done
