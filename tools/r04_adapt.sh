#!/bin/bash
# Round 4: the GPU suite (one process), then config 1 scaled / config 2 / config 4
# under ADAPT (CONFIGS), kernel times per launch.  Output under gpurun_out/$TAG.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/${TAG:-r04adapt}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${K:+-k "$K"} \
    > "$OUT/pytest_gpu.txt" 2>&1 || { tail -30 "$OUT/pytest_gpu.txt"; exit 1; }
  tail -2 "$OUT/pytest_gpu.txt"
fi
for c in ${CONFIGS:-1 4}; do
  case $c in
    1) args="--config 1 --mode adapt --steps 2 --warmup 1" ;;
    2) args="--mode adapt --no-adapt --steps 5 --warmup 2" ;;
    4) args="--config 4 --mode adapt --steps 2 --warmup 1" ;;
  esac
  timeout -k 10 300 python3 -u bench.py $args --no-cpu > "$OUT/c${c}a.json" 2> "$OUT/c${c}a.err" || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1].split('/')[-1], '%.3f ms' % d['ms_per_step'], d.get('batch_stats'), {n: round(v['avg_ms'] * 1e3, 2) for n, v in d['kernels'].items() if not n.startswith('_')})" "$OUT/c${c}a.json"
done
