#!/bin/bash
# Round-2 closing measurement set, after the batch-path launch fusions, on one
# box.  Part "run": GPU tests, smoke, the default bench (headline + CPU
# baseline), configs 3 / 4 (ADAPT) / 5.  Part "prof": config 2 / 3 rocprof
# kernel traces and the PMC passes behind bench.py's roofline.
# Usage: bash tools/r02c_final.sh run|prof
set -o pipefail
mkdir -p gpurun_out/r02c
if [[ $1 == run ]]; then
  bash tools/gpu_tests.sh || exit $?
  timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02c/smoke.txt 2>&1 || exit $?
  timeout -k 10 300 python3 -u bench.py > gpurun_out/r02c/bench_default.json 2> gpurun_out/r02c/bench_default.err || exit $?
  timeout -k 10 300 python3 -u bench.py --config 3 --steps 2 --warmup 1 --cpu-seconds 10 > gpurun_out/r02c/bench_config3.json 2> gpurun_out/r02c/bench_config3.err || exit $?
  timeout -k 10 400 python3 -u bench.py --config 4 --mode adapt --steps 2 --warmup 1 --no-cpu > gpurun_out/r02c/bench_config4_adapt.json 2> gpurun_out/r02c/bench_config4_adapt.err || exit $?
  timeout -k 10 400 python3 -u bench.py --config 5 --steps 1 --warmup 1 --no-cpu > gpurun_out/r02c/bench_config5.json 2> gpurun_out/r02c/bench_config5.err || exit $?
else
  bash tools/c2prof.sh r02c_c2 || exit $?
  bash tools/c3prof.sh r02c_c3 || exit $?
  TAG=r02c_pmc bash tools/pmc_roofline.sh > gpurun_out/r02c/pmc.log 2>&1
fi
