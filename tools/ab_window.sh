#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/abw
for r in 1 2; do
  for v in base w16 w32; do
    lib=$v; [ $v = base ] && lib=""
    KSIM_LIB_VARIANT=$lib timeout -k 10 300 python3 -u bench.py --config 4 --mode adapt --pods4 300000 --steps 1 --warmup 1 --no-cpu > gpurun_out/abw/c4_${v}_$r.json 2> gpurun_out/abw/c4_${v}_$r.err || exit $?
    KSIM_LIB_VARIANT=$lib timeout -k 10 200 python3 -u bench.py --mode adapt --steps 3 --warmup 1 --no-cpu > gpurun_out/abw/c2_${v}_$r.json 2> gpurun_out/abw/c2_${v}_$r.err || exit $?
  done
done
