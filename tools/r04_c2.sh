#!/bin/bash
# Round 4 A/B: config 2 (the default line) and the batch-path GPU tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/${TAG:-r04c2}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shard.py tests/test_gpu_batch_norm.py -m gpu -x -q \
  --timeout 200 --timeout-method thread -k "${K:-batch or lazy or replicated or config2}" > "$OUT/pytest.txt" 2>&1 || { tail -30 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
for i in 1 2; do
  timeout -k 10 300 python3 -u bench.py --no-cpu --no-adapt --steps 5 --warmup 2 > "$OUT/c2_$i.json" 2> "$OUT/c2_$i.err" || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1].split('/')[-1], '%.3f ms' % d['ms_per_step'], '%.3e' % d['value'], {n: round(v['avg_ms'] * 1e3, 2) for n, v in d['kernels'].items() if not n.startswith('_')})" "$OUT/c2_$i.json"
done
