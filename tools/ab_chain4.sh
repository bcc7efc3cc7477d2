#!/bin/bash
# Config 4 ADAPT A/B on one box: the chain fused into k_adapt_pairs (default)
# against the separate chain launch (KSIM_CHAIN_SEPARATE=1).
set -o pipefail
mkdir -p gpurun_out/abchain
for v in fused separate; do
  if [[ $v == separate ]]; then export KSIM_CHAIN_SEPARATE=1; else unset KSIM_CHAIN_SEPARATE; fi
  timeout -k 10 300 python3 -u bench.py --config 4 --mode adapt --steps 1 --warmup 1 --no-cpu > gpurun_out/abchain/c4a_$v.json 2> gpurun_out/abchain/c4a_$v.err || exit $?
done
