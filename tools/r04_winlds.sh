#!/bin/bash
# Round 4 A/B: the doubling window's rounds from LDS-staged rows (default) or
# global gathers (KSIM_WIN_GATHER=1), parity first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/${TAG:-r04winlds}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch_norm.py tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 200 --timeout-method thread -k "adapt or config1" > "$OUT/pytest.txt" 2>&1 || { tail -20 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
for v in lds; do
  if [ $v = gather ]; then export KSIM_WIN_GATHER=1; fi
  timeout -k 10 300 python3 -u bench.py --config 1 --mode adapt --steps 2 --warmup 1 --no-cpu > "$OUT/c1a_$v.json" 2> "$OUT/c1a_$v.err" || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1].split('/')[-1], '%.3f ms' % d['ms_per_step'], {n: round(v['avg_ms'] * 1e3, 2) for n, v in d['kernels'].items() if not n.startswith('_')})" "$OUT/c1a_$v.json"
done
