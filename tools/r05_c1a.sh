#!/bin/bash
# Round 5: config 1 under ADAPT after a change: its parity tests, the batch-end
# diagnostics and the bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/${TAG:-r05c1a}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_batch_norm.py tests/test_gpu_parity.py -m gpu -x -q -k "adapt or norm" \
  --timeout 300 --timeout-method thread > "$OUT/pytest.txt" 2>&1 || { tail -30 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
KSIM_LIB_VARIANT=adbg timeout -k 10 400 python3 -u tools/adapt_dbg.py > "$OUT/adbg.txt" 2>&1 || exit 1
tail -1 "$OUT/adbg.txt"
timeout -k 10 400 python3 -u bench.py --config 1 --mode adapt --steps 2 --warmup 1 --no-cpu > "$OUT/bench_c1a.json" 2> "$OUT/bench_c1a.err" || exit 1
python3 -c "
import json; d=json.loads(open('$OUT/bench_c1a.json').read().strip().splitlines()[-1])
print('config1 adapt', round(d['ms_per_step'],1), 'ms', d['batch_stats'], {k: round(v['avg_ms']*1e3,2) for k, v in d['kernels'].items() if not k.startswith('_')})"
