#!/bin/bash
# Config 5 (policy sweep) with 1, 2, 4 and 8 concurrent engines on one GPU.
set -o pipefail
mkdir -p gpurun_out/absw
for s in 1 2 4 8; do
  timeout -k 10 300 python3 -u bench.py --config 5 --sweep 128 --sweep-streams $s --steps 1 --warmup 1 --no-cpu > gpurun_out/absw/c5_s$s.json 2> gpurun_out/absw/c5_s$s.err || exit $?
done
