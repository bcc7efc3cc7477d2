#!/bin/bash
# Round 4 A/B: the doubling window's radix (KSIM_WIN_RADIX 4 / 8 / 16), parity first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/${TAG:-r04radix}
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in 16 8 4; do
  KSIM_WIN_RADIX=$r timeout -k 10 300 python -u -m pytest tests/test_gpu_batch_norm.py tests/test_gpu_parity.py -m gpu -x -q \
    --timeout 200 --timeout-method thread -k "adapt or config1" > "$OUT/pytest_$r.txt" 2>&1 || { tail -20 "$OUT/pytest_$r.txt"; exit 1; }
  echo "radix $r: $(tail -1 $OUT/pytest_$r.txt)"
  KSIM_WIN_RADIX=$r timeout -k 10 300 python3 -u bench.py --config 1 --mode adapt --steps 2 --warmup 1 --no-cpu > "$OUT/c1a_$r.json" 2> "$OUT/c1a_$r.err" || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1].split('/')[-1], '%.3f ms' % d['ms_per_step'], {n: round(v['avg_ms'] * 1e3, 2) for n, v in d['kernels'].items() if not n.startswith('_')})" "$OUT/c1a_$r.json"
done
