#!/bin/bash
# Round 3 measurement set (VERDICT r02 "Next round" 2): the default bench's
# rocprof kernel stats as CSV; SQ cycle / wait counters and the VALU
# instruction mix of the config-2 P100 batch kernels; FETCH / WRITE / VALU of
# the config-3 topology batch kernels and of the config-4 ADAPT kernels; the
# config-4 ADAPT bench line with its CPU baseline.  One rocprofv3 --pmc pass
# per counter group, each under its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/${TAG:-r03pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv -- \
  python3 -u bench.py --no-cpu > "$OUT/bench_stats.json" 2> "$OUT/bench_stats.err" || exit $?
find "$OUT/stats" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats_config2.csv" \;
head -8 "$OUT/kernel_stats_config2.csv"
pass() {  # label kernel-regex bench-args counters...
  local label=$1 kre=$2 args=$3; shift 3
  echo "== $label: $*"
  timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-include-regex "$kre" -d "$OUT/$label" -o run \
    --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-adapt $args > "$OUT/$label.log" 2>&1
  local rc=$?; if [ $rc -ne 0 ]; then echo "$label failed rc=$rc"; exit $rc; fi
}
pass c2_sq "k_batch" "" SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU
pass c2_mix "k_batch" "" SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU
pass c2_mem "k_batch" "" SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SMEM SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE
pass c2_fetch "k_batch" "" FETCH_SIZE
pass c3_fetch "k_tb_" "--config 3" FETCH_SIZE
pass c3_write "k_tb_" "--config 3" WRITE_SIZE
pass c3_sq "k_tb_" "--config 3" SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU
pass c4_fetch "k_adapt" "--config 4 --mode adapt --pods4 100000" FETCH_SIZE
pass c4_write "k_adapt" "--config 4 --mode adapt --pods4 100000" WRITE_SIZE
pass c4_sq "k_adapt" "--config 4 --mode adapt --pods4 100000" SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU
python3 tools/pmc_table.py "$OUT" > "$OUT/summary.txt" && cat "$OUT/summary.txt"
timeout -k 10 400 python3 -u bench.py --config 4 --mode adapt --steps 2 --warmup 1 > "$OUT/bench_config4_adapt.json" \
  2> "$OUT/bench_config4_adapt.err" || exit $?
tail -c 600 "$OUT/bench_config4_adapt.json"
