#!/bin/bash
# A/B of the batch merge: register merge (default) against the LDS merge
# (KSIM_MERGE_LDS=1), alternating, after the GPU parity tests.
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/${TAG:-ab}
mkdir -p "$OUT"
cd "${GRAFT_REPO_ROOT:-.}"
step() { echo "== $*" >&2 ; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
for i in 1 2; do
  step timeout -k 10 200 python -u bench.py --no-cpu --no-adapt > "$OUT/reg_$i.json" 2>> "$OUT/bench.err"
  KSIM_MERGE_LDS=1 step timeout -k 10 200 python -u bench.py --no-cpu --no-adapt > "$OUT/lds_$i.json" 2>> "$OUT/bench.err"
done
export TMPDIR=/tmp
step timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu > "$OUT/prof.log" 2>&1
echo done
