#!/bin/bash
# Round 4: topology batches across classes, replicated topology batches, the
# doubling ADAPT window: their GPU tests, then config 3, config 1 scaled under
# ADAPT (doubling) and the drop-in cycle.  Output under
# gpurun_out/${TAG:-r04next}.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/${TAG:-r04next}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu_tbatch.py tests/test_gpu_shard.py tests/test_gpu_parity.py \
    tests/test_gpu_fw.py tests/test_gpu_batch_norm.py -m gpu -x -v --timeout 200 --timeout-method thread \
    -k "${K:-tbatch or config3 or cross or app or fill or mixed or weights or timing or fw or replicated or adapt or config1}" \
    > "$OUT/pytest.txt" 2>&1 || { tail -40 "$OUT/pytest.txt"; exit 1; }
  tail -3 "$OUT/pytest.txt"
fi
summ() {
  python3 - "$1" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = {n: round(v['avg_ms'] * 1e3, 2) for n, v in d.get('kernels', {}).items() if not n.startswith('_')}
print(sys.argv[1].split('/')[-1], '%.3f ms' % d['ms_per_step'], d.get('batch_stats'), ks)
PY
}
timeout -k 10 400 python3 -u bench.py --config 3 --steps 3 --warmup 1 > "$OUT/bench_config3.json" 2> "$OUT/bench_config3.err" || exit $?
summ "$OUT/bench_config3.json"
timeout -k 10 300 python3 -u bench.py --config 1 --mode adapt --steps 2 --warmup 1 --no-cpu > "$OUT/c1a_dbl.json" 2> "$OUT/c1a_dbl.err" || exit $?
summ "$OUT/c1a_dbl.json"
[ -n "$NOFW" ] && exit 0
timeout -k 10 300 python3 -u bench.py --mode fw > "$OUT/fw.json" 2> "$OUT/fw.err" || exit $?
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); [print(r['nodes'], round(r['engine']['us_per_cycle'],1), {k: round(v,1) for k,v in r['engine']['us_per_call'].items()}, round(r['oracle_cpu_1thread']['us_per_cycle'],1)) for r in d['rows']]" "$OUT/fw.json"
