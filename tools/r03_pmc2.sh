#!/bin/bash
# Round 3: chain + pairs phase clocks (cpclk flavor), then PMC passes of the
# deferred-commit kernels (config 2 P100: k_batch_top_commit / chain_pairs;
# config 4 ADAPT: k_adapt_*), one rocprofv3 --pmc pass per counter group.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/${TAG:-r03pmc2}
mkdir -p "$OUT"
export TMPDIR=/tmp
KSIM_LIB_VARIANT=cpclk timeout -k 10 200 python3 -u tools/cp_clocks.py > "$OUT/cp_clocks.txt" 2>&1 || exit $?
cat "$OUT/cp_clocks.txt"
pass() {  # label kernel-regex bench-args counters...
  local label=$1 kre=$2 args=$3; shift 3
  echo "== $label: $*"
  timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-include-regex "$kre" -d "$OUT/$label" -o run \
    --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-adapt $args > "$OUT/$label.log" 2>&1
  local rc=$?; if [ $rc -ne 0 ]; then echo "$label failed rc=$rc"; exit $rc; fi
}
pass c2_sq "k_batch" "" SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU
pass c2_mix "k_batch" "" SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_LDS
pass c2_fetch "k_batch" "" FETCH_SIZE
pass c2_write "k_batch" "" WRITE_SIZE
pass c4_fetch "k_adapt" "--config 4 --mode adapt --pods4 100000" FETCH_SIZE
pass c4_write "k_adapt" "--config 4 --mode adapt --pods4 100000" WRITE_SIZE
pass c4_sq "k_adapt" "--config 4 --mode adapt --pods4 100000" SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU
python3 tools/pmc_table.py "$OUT" > "$OUT/summary.txt" && cat "$OUT/summary.txt"
