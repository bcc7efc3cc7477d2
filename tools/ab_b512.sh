#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/ab512
for v in "" b512t8 b512t16; do
  KSIM_LIB_VARIANT=$v timeout -k 10 200 python3 -u bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/ab512/c2_${v:-base}.json 2> gpurun_out/ab512/c2_${v:-base}.err || exit $?
  KSIM_LIB_VARIANT=$v timeout -k 10 200 python3 -u bench.py --config 4 --mode adapt --pods4 200000 --steps 2 --warmup 1 --no-cpu > gpurun_out/ab512/c4a_${v:-base}.json 2> gpurun_out/ab512/c4a_${v:-base}.err || exit $?
done
