#!/bin/bash
# Round 4 check on one box: every -m gpu test (one process), smoke, the
# default bench line.  Output under gpurun_out/${TAG:-r04check}.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/${TAG:-r04check}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${K:+-k "$K"} \
  > "$OUT/pytest_gpu.txt" 2>&1 || { tail -30 "$OUT/pytest_gpu.txt"; exit 1; }
tail -3 "$OUT/pytest_gpu.txt"
[ -n "$NOSMOKE" ] && exit 0
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.txt" 2>&1 || exit $?
tail -1 "$OUT/smoke.txt"
timeout -k 10 400 python3 -u bench.py ${BENCH_ARGS} > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || exit $?
tail -c 600 "$OUT/bench_default.json"; echo
