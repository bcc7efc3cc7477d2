#!/bin/bash
# Config 2 (P100 headline + ADAPT line) A/B on one box: default library against
# KSIM_LIB_VARIANT flavors, REPS times interleaved.
set -o pipefail
mkdir -p gpurun_out/abc2
for r in $(seq 1 ${REPS:-1}); do
  for v in base "$@"; do
    lib=$v; [[ $v == base ]] && lib=""
    KSIM_LIB_VARIANT=$lib timeout -k 10 200 python3 -u bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/abc2/c2_${v}_$r.json 2> gpurun_out/abc2/c2_${v}_$r.err || exit $?
  done
done
