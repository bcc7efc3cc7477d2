#!/bin/bash
# Round 3 first GPU call: framework-driven compat tests, then SQ counters.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/r03a
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_fw.py -x -v --timeout 240 --timeout-method thread > "$OUT/pytest_fw.log" 2>&1
rc=$?; tail -5 "$OUT/pytest_fw.log"; if [ $rc -ne 0 ]; then exit $rc; fi
TAG=r03sq bash tools/r03_sq.sh
