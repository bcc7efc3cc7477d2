#!/bin/bash
# Config 2 A/B on one box: the ADAPT window scan fused into k_adapt_top (default)
# against the separate one-block window scan (KSIM_WINDOW_SEPARATE=1), REPS times interleaved.
set -o pipefail
mkdir -p gpurun_out/abwin
for r in $(seq 1 ${REPS:-3}); do
  for v in fused separate; do
    if [[ $v == separate ]]; then export KSIM_WINDOW_SEPARATE=1; else unset KSIM_WINDOW_SEPARATE; fi
    timeout -k 10 200 python3 -u bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/abwin/c2_${v}_$r.json 2> gpurun_out/abwin/c2_${v}_$r.err || exit $?
  done
done
