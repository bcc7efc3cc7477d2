#!/bin/bash
# Config 3 with and without the persistent domain tables (same box).
set -o pipefail
mkdir -p gpurun_out/abp
timeout -k 10 300 python3 -u bench.py --config 3 --steps 1 --warmup 1 --no-cpu > gpurun_out/abp/c3_ptab.json 2> gpurun_out/abp/c3_ptab.err || exit $?
KSIM_NO_PTAB=1 timeout -k 10 300 python3 -u bench.py --config 3 --steps 1 --warmup 1 --no-cpu > gpurun_out/abp/c3_noptab.json 2> gpurun_out/abp/c3_noptab.err
