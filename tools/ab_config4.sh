set -o pipefail
for v in tiles top; do
  unset KSIM_BATCH_TILES; [ $v = tiles ] && export KSIM_BATCH_TILES=1
  timeout -k 10 400 python3 -u bench.py --config 4 --pods4 200000 --steps 1 --warmup 1 --no-cpu > gpurun_out/ab4_$v.json 2> gpurun_out/ab4_$v.err || exit $?
  python3 -c "
import json
d=json.loads(open('gpurun_out/ab4_$v.json').read().strip().splitlines()[-1])
print('$v', 'value %.4e'%d['value'], 'ms/step %.3f'%d['ms_per_step'], d['batch_stats'], {k:(round(x['avg_ms']*1000,2)) for k,x in d['kernels'].items()}, 'eval %.2f us'%(d['roofline']['avg_launch_ms']*1000))
"
done
