#!/bin/bash
# Config-2 batch path on the box: kernel trace + stats of the bench (no CPU leg).
# Usage: bash tools/c2prof.sh [tag] [extra bench args]
set -o pipefail
T=${1:-c2}
shift
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof -o $T -- python3 bench.py --steps 5 --warmup 2 --no-cpu "$@" > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err
