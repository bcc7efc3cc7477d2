#!/bin/bash
# ADAPT A/B on one box (config 2 ADAPT line, config 4 ADAPT on 200k pods),
# default library against flavors, REPS times interleaved.
set -o pipefail
mkdir -p gpurun_out/aba
for r in $(seq 1 ${REPS:-1}); do
  for v in base "$@"; do
    lib=$v; [[ $v == base ]] && lib=""
    KSIM_LIB_VARIANT=$lib timeout -k 10 200 python3 -u bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/aba/c2_${v}_$r.json 2> gpurun_out/aba/c2_${v}_$r.err || exit $?
    KSIM_LIB_VARIANT=$lib timeout -k 10 200 python3 -u bench.py --config 4 --mode adapt --pods4 200000 --steps 2 --warmup 1 --no-cpu > gpurun_out/aba/c4a_${v}_$r.json 2> gpurun_out/aba/c4a_${v}_$r.err || exit $?
  done
done
