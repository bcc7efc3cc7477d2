#!/bin/bash
# Bench the headline (config 2) and the other configs on one box, one JSON per config.
# Usage: TAG=name bash tools/bench_all.sh [configs...]   (default: 2 3)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-bench}
mkdir -p "$OUT"
for c in ${@:-2 3}; do
  case $c in
    2) args="--steps 10 --warmup 3" ;;
    2a) args="--steps 10 --warmup 3 --mode adapt --no-adapt" ;;
    3) args="--config 3 --steps 3 --warmup 1 --pods3 4000" ;;
    4) args="--config 4 --steps 1 --warmup 1 --pods4 200000" ;;
    5) args="--config 5 --steps 1 --warmup 1 --sweep 64" ;;
  esac
  timeout -k 10 400 python3 -u bench.py $args --cpu-seconds 5 > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err" || exit $?
  tail -c 400 "$OUT/bench_$c.json"; echo
done
