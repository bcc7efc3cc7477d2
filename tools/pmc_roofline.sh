#!/bin/bash
# PMC passes behind bench.py's roofline: HBM traffic (FETCH_SIZE, WRITE_SIZE)
# and the vector / scalar instruction counts of the evaluation kernel, one
# rocprofv3 pass per counter group (kernel trace only), for config 2
# (k_batch_top) and config 3 (k_filter_score).  Output: gpurun_out/$TAG/*,
# summarised by tools/pmc_roofline.py into traffic.json / valu.json entries.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${TAG:-pmc_roof}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
pass() {  # label, kernel regex, pass, bench args, counters...
  local label=$1 kre=$2 p=$3 args=$4; shift 4
  echo "== $label $p: $*"
  timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-include-regex "$kre" -d "$OUT/$label/$p" -o run \
    --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-adapt $args > "$OUT/$label.$p.log" 2>&1
  local rc=$?; if [ $rc -ne 0 ]; then echo "$label $p failed rc=$rc"; return $rc; fi
}
for spec in "config2|k_batch_top|" "config3|k_filter_score|--config 3 --pods3 600"; do
  IFS='|' read -r label kre args <<< "$spec"
  pass $label $kre fetch "$args" FETCH_SIZE || exit $?
  pass $label $kre write "$args" WRITE_SIZE || exit $?
  pass $label $kre sq "$args" SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VALU_FP64 SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY || exit $?
done
python3 tools/pmc_roofline.py "$OUT" > "$OUT/summary.json" && cat "$OUT/summary.json"
