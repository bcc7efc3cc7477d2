#!/bin/bash
# Round 4 topology batches across class conflicts: the topology batch and
# config-3 parity tests, the drop-in call tests, then the config-3 bench line.
# Output under gpurun_out/${TAG:-r04tb}.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/${TAG:-r04tb}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_tbatch.py tests/test_gpu_shard.py tests/test_gpu_parity.py \
  tests/test_gpu_fw.py -m gpu -x -v --timeout 200 --timeout-method thread \
  -k "${K:-tbatch or config3 or cross or app or fill or mixed or weights or timing or fw or replicated}" \
  > "$OUT/pytest.txt" 2>&1 || { tail -40 "$OUT/pytest.txt"; exit 1; }
tail -3 "$OUT/pytest.txt"
timeout -k 10 400 python3 -u bench.py --config 3 --steps 3 --warmup 1 ${BENCH_ARGS} > "$OUT/bench_config3.json" 2> "$OUT/bench_config3.err" || exit $?
python3 - "$OUT/bench_config3.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print({k: d.get(k) for k in ("value", "ms_per_step", "unit")})
print({k: d.get(k) for k in ("roofline", "stats", "vs_cpu")})
PY
[ -n "$NOFW" ] && exit 0
timeout -k 10 300 python3 -u bench.py --mode fw > "$OUT/fw.json" 2> "$OUT/fw.err" || exit $?
tail -c 1500 "$OUT/fw.json"; echo
