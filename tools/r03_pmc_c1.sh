#!/bin/bash
# Round 3: PMC passes of config 1 scaled (the static-class STAB kernels
# k_batch_top / k_batch_chain_pairs / k_batch_commit), one rocprofv3 --pmc pass
# per counter group, kernel trace only.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/${TAG:-r03pmc_c1}
mkdir -p "$OUT"
export TMPDIR=/tmp
pass() {  # label kernel-regex bench-args counters...
  local label=$1 kre=$2 args=$3; shift 3
  echo "== $label: $*"
  timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-include-regex "$kre" -d "$OUT/$label" -o run \
    --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-adapt $args > "$OUT/$label.log" 2>&1
  local rc=$?; if [ $rc -ne 0 ]; then echo "$label failed rc=$rc"; exit $rc; fi
}
pass c1_sq "k_batch" "--config 1" SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU
pass c1_mix "k_batch" "--config 1" SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_LDS
pass c1_fetch "k_batch" "--config 1" FETCH_SIZE
pass c1_write "k_batch" "--config 1" WRITE_SIZE
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv -- \
  python3 bench.py --config 1 --steps 3 --warmup 1 --no-cpu > "$OUT/bench_rocprof.json" 2> "$OUT/bench_rocprof.err" || exit $?
find "$OUT/stats" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats_config1.csv" \;
python3 tools/pmc_table.py "$OUT" > "$OUT/pmc_summary.txt" && cat "$OUT/pmc_summary.txt"
