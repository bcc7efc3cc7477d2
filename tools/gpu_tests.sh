#!/bin/bash
# GPU parity run on the box: every -m gpu test, one process, then smoke.
# Usage (from the repo root on the GPU box): bash tools/gpu_tests.sh [pytest -k expr]
set -o pipefail
mkdir -p gpurun_out
K=${1:+-k "$1"}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread $K \
  > gpurun_out/pytest_gpu.txt 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.txt
exit $rc
