#!/bin/bash
# Config 3 A/B on one box, each variant REPS times interleaved.  A variant is a
# KSIM_LIB_VARIANT flavor, or ENV=1 to run the default library with that
# environment variable set.  Usage: REPS=2 bash tools/ab_c3.sh head KSIM_NO_PTAB=1
set -o pipefail
mkdir -p gpurun_out/abc3
for r in $(seq 1 ${REPS:-1}); do
  for v in base "$@"; do
    if [[ $v == *=* ]]; then envs=("$v"); lib=""; else envs=(); lib=$v; fi
    [[ $v == base ]] && lib=""
    tag=${v//=/_}
    env "${envs[@]}" KSIM_LIB_VARIANT=$lib timeout -k 10 300 python3 -u bench.py --config 3 --steps 1 --warmup 1 --no-cpu --pods3 4000 > gpurun_out/abc3/c3_${tag}_$r.json 2> gpurun_out/abc3/c3_${tag}_$r.err || exit $?
  done
done
