set -o pipefail
mkdir -p gpurun_out/r03adtop
for r in 1 2; do
for v in wide narrow; do
  if [ $v == narrow ]; then export KSIM_ADAPT_TOP_NARROW=1; else unset KSIM_ADAPT_TOP_NARROW; fi
  timeout -k 10 300 python3 -u bench.py --config 1 --mode adapt --steps 2 --warmup 1 --no-cpu > gpurun_out/r03adtop/c1a_${v}_$r.json 2> gpurun_out/r03adtop/c1a_${v}_$r.err || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1].split('/')[-1], '%.3f ms' % d['ms_per_step'], {n: round(v['avg_ms'] * 1e3, 2) for n, v in d['kernels'].items() if not n.startswith('_')})" gpurun_out/r03adtop/c1a_${v}_$r.json
done
done
