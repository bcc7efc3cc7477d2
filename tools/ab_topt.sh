#!/bin/bash
# A/B of the top-T list length at B = 256 (config 2, P100 + ADAPT).
set -o pipefail
mkdir -p gpurun_out/abt
for v in "" b256t12 b256t16; do
  KSIM_LIB_VARIANT=$v timeout -k 10 200 python3 -u bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/abt/c2_${v:-base}.json 2> gpurun_out/abt/c2_${v:-base}.err || exit $?
done
