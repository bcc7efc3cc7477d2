#!/bin/bash
# Round 4 A/B: config 1 scaled (P100, generic batch top) and its batch tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/${TAG:-r04c1}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch_norm.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 \
  --timeout-method thread > "$OUT/pytest.txt" 2>&1 || { tail -30 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
for c in 1 1b; do
  case $c in
    1) args="--config 1 --steps 3 --warmup 1 --no-cpu" ;;
    1b) args="--config 1 --steps 3 --warmup 1 --no-cpu" ;;
  esac
  timeout -k 10 300 python3 -u bench.py $args > "$OUT/c$c.json" 2> "$OUT/c$c.err" || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1].split('/')[-1], '%.3f ms' % d['ms_per_step'], {n: round(v['avg_ms'] * 1e3, 2) for n, v in d['kernels'].items() if not n.startswith('_')})" "$OUT/c$c.json"
done
