#!/bin/bash
# Round 3 re-entry: the whole -m gpu suite on the current tree, smoke, the
# default bench line, and the rocprof kernel stats of the same command.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/${TAG:-r03full}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1
rc=$?; tail -3 "$OUT/pytest_gpu.txt"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.txt" 2>&1 || exit $?
timeout -k 10 400 python3 -u bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || exit $?
tail -1 "$OUT/bench_default.json"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 -u bench.py --no-cpu > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err" || exit $?
find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
head -12 "$OUT/kernel_stats.csv"
