#!/bin/bash
# Round 5: the drop-in cycle under rocprofv3 kernel + HIP runtime traces
# (API call and kernel durations of bench.py --mode fw).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/${TAG:-r05fwtrace}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --hip-runtime-trace --stats -d "$OUT/prof" -o fw --output-format csv -- \
  python3 bench.py --mode fw > "$OUT/bench_fw.json" 2> "$OUT/bench_fw.err" || exit $?
for f in $(find "$OUT/prof" -name '*_stats.csv'); do cp "$f" "$OUT/"; done
rm -rf "$OUT/prof"
ls "$OUT"
head -25 "$OUT"/*hip_api_stats.csv | cut -c1-150
head -12 "$OUT"/*kernel_stats.csv | cut -c1-150
