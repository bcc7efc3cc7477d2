#!/bin/bash
# Round 4 A/B: config 3 topology batch run rules (KSIM_TB_NOCROSS: runs end at
# every class conflict, round 3; KSIM_TB_CAP: run length cap).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/${TAG:-r04tbcap}
mkdir -p "$OUT"
export TMPDIR=/tmp
summ() {
  python3 - "$1" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = {n: round(v['avg_ms'] * 1e3, 2) for n, v in d.get('kernels', {}).items() if not n.startswith('_')}
print(sys.argv[1].split('/')[-1], '%.3f ms' % d['ms_per_step'], d.get('batch_stats'), ks)
PY
}
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch_norm.py tests/test_gpu_parity.py -m gpu -x -v --timeout 200 \
  --timeout-method thread -k "adapt or config1" > "$OUT/pytest_adapt.txt" 2>&1 || { tail -30 "$OUT/pytest_adapt.txt"; exit 1; }
tail -1 "$OUT/pytest_adapt.txt"
timeout -k 10 300 python3 -u bench.py --config 1 --mode adapt --steps 2 --warmup 1 --no-cpu > "$OUT/c1a.json" 2> "$OUT/c1a.err" || exit $?
summ "$OUT/c1a.json"
for v in "KSIM_TB_NOCROSS=1" "KSIM_TB_CAP=10" "KSIM_TB_CAP=12" "KSIM_TB_CAP=16" "KSIM_TB_CAP=24"; do
  tag=$(echo $v | tr '=' '_')
  env $v timeout -k 10 300 python3 -u bench.py --config 3 --steps 2 --warmup 1 --no-cpu > "$OUT/c3_$tag.json" 2> "$OUT/c3_$tag.err" || exit $?
  summ "$OUT/c3_$tag.json"
done
