#!/bin/bash
# rocprofv3 kernel stats of the config 4 ADAPT line (one step), beside the
# line's own per-kernel event times.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/${TAG:-r04rocprof4}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv -- \
  python3 -u bench.py --config 4 --mode adapt --steps 1 --warmup 1 --no-cpu > "$OUT/bench_config4a.json" 2> "$OUT/bench.err" || exit $?
find "$OUT/stats" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats_config4a.csv" \;
rm -rf "$OUT/stats"
head -8 "$OUT/kernel_stats_config4a.csv"
