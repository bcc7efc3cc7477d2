#!/bin/bash
# Round 5 A/B of library flavors on config 2 (P100, no CPU leg): bench line and
# phase clocks per flavor.  VARIANTS="base u2" CLK="tcclk u2clk" bash tools/r05_ab.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/${TAG:-r05ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in ${VARIANTS:-base}; do
  vv=$v; [ "$v" = base ] && vv=""
  if [ -n "$PARITY" ]; then
    KSIM_LIB_VARIANT=$vv timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "batch" \
      --timeout 200 --timeout-method thread > "$OUT/pytest_$v.txt" 2>&1 || { tail -20 "$OUT/pytest_$v.txt"; exit 1; }
    echo "$v: $(tail -1 $OUT/pytest_$v.txt)"
  fi
  for rep in 1 2; do
    KSIM_LIB_VARIANT=$vv timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu --no-adapt ${BENCH_ARGS} > "$OUT/bench_${v}_$rep.json" 2> "$OUT/bench_${v}_$rep.err" || exit $?
    python3 -c "
import json,sys; d=json.loads(open('$OUT/bench_${v}_$rep.json').read().strip().splitlines()[-1])
print('$v', round(d['ms_per_step'],3), 'ms', d['batch_stats']['batches'], {k: round(v['avg_ms_events']*1e3,2) for k, v in d['kernels'].items() if not k.startswith('_')}, 'b2b', round(d['roofline']['avg_launch_ms']*1e3,2))"
  done
done
for v in ${CLK}; do
  KSIM_LIB_VARIANT=$v timeout -k 10 150 python3 -u tools/tc_clocks.py > "$OUT/clk_$v.txt" 2>&1 || exit $?
  echo "$v: $(cat $OUT/clk_$v.txt)"
done
