set -o pipefail
mkdir -p gpurun_out/r05r
export TMPDIR=/tmp
KSIM_LIB_VARIANT=adbg timeout -k 10 400 python3 -u tools/adapt_dbg.py > gpurun_out/r05r/adbg.txt 2>&1; cat gpurun_out/r05r/adbg.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_shard.py -m gpu -x -q -k "replicated_config4" --timeout 300 --timeout-method thread > gpurun_out/r05r/pytest.txt 2>&1; tail -2 gpurun_out/r05r/pytest.txt
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/r05r/prof4 -o c4 -- python3 -u bench.py --config 4 --steps 2 --warmup 1 --no-cpu > gpurun_out/r05r/bench_c4.json 2> gpurun_out/r05r/bench_c4.err || exit 1
python3 tools/kstats.py $(find gpurun_out/r05r/prof4 -name "*results.db" | head -1) | head -6
python3 -c "
import json; d=json.loads(open('gpurun_out/r05r/bench_c4.json').read().strip().splitlines()[-1])
print(round(d['ms_per_step'],1), 'ms', '%.3e' % d['value'], d['batch_stats'], {k: round(v['avg_ms']*1e3,2) for k, v in d['kernels'].items() if not k.startswith('_')})"
