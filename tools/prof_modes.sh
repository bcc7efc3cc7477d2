#!/bin/bash
# rocprofv3 kernel-trace summaries of the per-pod path (ADAPT, config 3) and
# the batch path (config 2), one run each, under gpurun_out/$TAG/prof_*.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/${TAG:-run}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local name=$1; shift
  echo "== $name" >&2
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$name" -o run --output-format csv \
      -- python3 bench.py --no-cpu --steps 1 --warmup 0 "$@" > "$OUT/prof_$name.log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "profile $name failed rc=$rc"; exit $rc; fi
  python3 tools/trace_summary.py "$OUT/prof_$name/"*kernel_trace.csv > "$OUT/prof_$name.txt" 2>&1 || true
}
run batch
run adapt --mode adapt --pods 5000
run c3 --config 3 --pods3 2000
echo done
