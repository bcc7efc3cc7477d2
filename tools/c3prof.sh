#!/bin/bash
# Config-3 per-pod path on the box: kernel trace + stats of one bench step.
# Usage: bash tools/c3prof.sh [tag]
set -o pipefail
T=${1:-c3}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof -o $T -- python3 bench.py --config 3 --steps 1 --warmup 1 --no-cpu > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err
