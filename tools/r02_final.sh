#!/bin/bash
# Round-2 measurement set on one box: GPU tests, default bench (headline +
# CPU baseline), config 3, config 4 ADAPT, config 2 / 3 rocprof kernel traces.
set -o pipefail
mkdir -p gpurun_out/r02f
bash tools/gpu_tests.sh || exit $?
timeout -k 10 300 python3 -u bench.py > gpurun_out/r02f/bench_default.json 2> gpurun_out/r02f/bench_default.err || exit $?
timeout -k 10 300 python3 -u bench.py --config 3 --steps 2 --warmup 1 --cpu-seconds 10 > gpurun_out/r02f/bench_config3.json 2> gpurun_out/r02f/bench_config3.err || exit $?
timeout -k 10 400 python3 -u bench.py --config 4 --mode adapt --steps 2 --warmup 1 --no-cpu > gpurun_out/r02f/bench_config4_adapt.json 2> gpurun_out/r02f/bench_config4_adapt.err || exit $?
bash tools/c2prof.sh r02f_c2 || exit $?
bash tools/c3prof.sh r02f_c3
