#!/bin/bash
# One GPU call: parity tests, bench, rocprofv3 kernel stats.  Each GPU step has
# its own time limit; the script stops at the first failing step.
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/${TAG:-run}
mkdir -p "$OUT"
cd "${GRAFT_REPO_ROOT:-.}"
step() { echo "== $*" >&2 ; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
if [ -z "$NO_TESTS" ]; then
  step timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
fi
step timeout -k 10 300 python -u bench.py ${BENCH_ARGS} > "$OUT/bench.json" 2> "$OUT/bench.err"
if [ -z "$NO_PROF" ]; then
  export TMPDIR=/tmp
  step timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu > "$OUT/prof.log" 2>&1
fi
echo done
