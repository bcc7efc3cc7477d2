#!/bin/bash
# Round 3: SQ cycle counters (wave / busy cycles, waits) of the config-2 batch
# kernels, P100 and ADAPT, one rocprofv3 --pmc pass per group.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/${TAG:-r03sq}
mkdir -p "$OUT"
export TMPDIR=/tmp
pass() {  # label kre args counters...
  local label=$1 kre=$2 args=$3; shift 3
  echo "== $label: $*"
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "$kre" -d "$OUT/$label" -o run \
    --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-adapt $args > "$OUT/$label.log" 2>&1
  local rc=$?; if [ $rc -ne 0 ]; then echo "$label failed rc=$rc"; exit $rc; fi
}
pass p100_a "k_batch" "" SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU
pass p100_b "k_batch" "" SQ_INST_CYCLES_VMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM GRBM_GUI_ACTIVE
pass adapt_a "k_adapt" "--mode adapt" SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU
pass adapt_f "k_adapt" "--mode adapt" FETCH_SIZE
pass adapt_w "k_adapt" "--mode adapt" WRITE_SIZE
python3 tools/pmc_table.py "$OUT" > "$OUT/summary.txt" && cat "$OUT/summary.txt"
