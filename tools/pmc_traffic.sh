#!/bin/bash
# HBM traffic of the evaluation kernel from rocprofv3 PMC counters: one pass per
# counter group (FETCH_SIZE uses 3 TCC slots, WRITE_SIZE 2: never together), kernel
# trace only, no other trace domains.  Output: gpurun_out/$TAG/pmc/*.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/${TAG:-run}/pmc
mkdir -p "$OUT"
export TMPDIR=/tmp
KRE=${KRE:-k_batch_top_commit}
i=0
for C in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  echo "== pass $i: $C"
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "$KRE" -d "$OUT/p$i" -o run --output-format csv \
      -- python3 bench.py --steps 1 --warmup 0 --no-cpu ${BENCH_ARGS} > "$OUT/p$i.log" 2>&1
  rc=$?; if [ $rc -ne 0 ]; then echo "pass $i failed rc=$rc"; exit $rc; fi
done
python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.json" && cat "$OUT/summary.json"
