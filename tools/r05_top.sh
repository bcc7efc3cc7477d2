#!/bin/bash
# Round 5: the headline kernel after a change: the P100 / replicated parity
# tests, config 2's bench line (no CPU leg), its phase clocks and a rocprof
# summary.  Output under gpurun_out/${TAG}.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/${TAG:-r05top}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shard.py tests/test_gpu_stab.py -m gpu -x -q \
  --timeout 200 --timeout-method thread ${K:+-k "$K"} > "$OUT/pytest.txt" 2>&1 || { tail -30 "$OUT/pytest.txt"; exit 1; }
tail -2 "$OUT/pytest.txt"
timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu --no-adapt > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
python3 -c "
import json,sys; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print('config2', round(d['ms_per_step'],3), 'ms', d['batch_stats'], {k: round(v['avg_ms']*1e3,2) for k, v in d['kernels'].items() if not k.startswith('_')})"
KSIM_LIB_VARIANT=tcclk timeout -k 10 150 python3 -u tools/tc_clocks.py > "$OUT/tcclk.txt" 2>&1 || exit $?
cat "$OUT/tcclk.txt"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o c2 -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-adapt > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err" || exit $?
python3 tools/kstats.py $(find "$OUT/prof" -name '*results.db' | head -1) | head -6
