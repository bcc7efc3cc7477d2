#!/bin/bash
# Round 5 PMC passes for the bench lines' by-time dominant kernels (configs in
# CONFIGS: c1 P100, c1a ADAPT, c2 default, c3, c4a ADAPT, c5 sweep), one
# rocprofv3 --pmc pass per counter group (kernel trace only), then
# tools/pmc_entries.py folds them into profiles/valu.json / traffic.json.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/${TAG:-r05pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
pass() {  # label bench-args counters...
  local label=$1 args=$2; shift 2
  echo "== $label: $*"
  timeout -s KILL 200 rocprofv3 --pmc "$@" --kernel-include-regex "k_" -d "$OUT/$label" -o run \
    --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-adapt $args > "$OUT/$label.log" 2>&1
  local rc=$?; if [ $rc -ne 0 ]; then echo "$label failed rc=$rc"; tail -5 "$OUT/$label.log"; exit $rc; fi
}
for c in ${CONFIGS:-c1 c1a c3 c4a c5}; do
  case $c in
    c1) args="--config 1" ;;
    c1a) args="--config 1 --mode adapt" ;;
    c2) args="" ;;
    c2a) args="--mode adapt" ;;
    c3) args="--config 3" ;;
    c4) args="--config 4 --pods4 100000" ;;
    c4a) args="--config 4 --mode adapt --pods4 100000" ;;
    c5) args="--config 5 --sweep 16" ;;
  esac
  pass ${c}_sq "$args" SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU
  pass ${c}_fetch "$args" FETCH_SIZE
  pass ${c}_write "$args" WRITE_SIZE
done
python3 tools/pmc_table.py "$OUT" > "$OUT/summary.txt" && python3 tools/pmc_entries.py "$OUT" --box > "$OUT/entries.log" || exit 1
rm -rf "$OUT"/c*_sq "$OUT"/c*_fetch "$OUT"/c*_write      # the raw CSVs exceed what gpurun copies back
tail -3 "$OUT/entries.log"
