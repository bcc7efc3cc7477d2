#!/bin/bash
# Round 4: rocprofv3 kernel statistics of the secondary bench lines (config 3,
# config 1 ADAPT, config 4 ADAPT), next to their JSON lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/${TAG:-r04rocprof}
mkdir -p "$OUT"
export TMPDIR=/tmp
for c in 3 1a 4a; do
  case $c in
    3) args="--config 3 --steps 2 --warmup 1" ;;
    1a) args="--config 1 --mode adapt --steps 2 --warmup 1" ;;
    4a) args="--config 4 --mode adapt --steps 1 --warmup 1" ;;
  esac
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/stats_$c" -o run --output-format csv -- \
    python3 -u bench.py $args --no-cpu > "$OUT/bench_config$c.json" 2> "$OUT/bench_config$c.err" || exit $?
  find "$OUT/stats_$c" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats_config$c.csv" \;
  rm -rf "$OUT/stats_$c"
  head -8 "$OUT/kernel_stats_config$c.csv" | cut -c1-160
done
