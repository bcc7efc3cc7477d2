#!/bin/bash
# SQ counters of the per-pod cycle kernels on config 3 (tools/c3clk.py, 1500
# pods): instruction mix per wave.  Two PMC passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/${TAG:-pmc_c3}
mkdir -p "$OUT"
KRE='k_filter_score|k_topo_prefilter|k_select|k_bind'
run() {  # pass, counters...
  local pass=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "$KRE" -d "$OUT/$pass" -o run \
    --output-format csv -- python3 tools/c3clk.py 1500 > "$OUT/$pass.log" 2>&1
}
run p1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY || exit $?
run p2 SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE || exit $?
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections, statistics
acc = collections.defaultdict(list)
for f in glob.glob(f"{sys.argv[1]}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), x in sorted(acc.items()):
    print(f"{k[-40:]:40s} {c:22s} n={len(x):5d} median={statistics.median(x):14.1f}")
PY
