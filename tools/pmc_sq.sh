#!/bin/bash
# Instruction mix of one kernel from SQ counters (one rocprofv3 --pmc pass of
# <= 8 SQ counters, kernel trace only).  KRE = kernel regex, BENCH_ARGS for bench.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/${TAG:-run}/sq
mkdir -p "$OUT"
export TMPDIR=/tmp
KRE=${KRE:-k_batch_top_commit}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY \
    --kernel-include-regex "$KRE" -d "$OUT/p1" -o run --output-format csv \
    -- python3 bench.py --steps 1 --warmup 0 --no-cpu ${BENCH_ARGS} > "$OUT/p1.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FP64 SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_WAIT_ANY GRBM_GUI_ACTIVE \
    --kernel-include-regex "$KRE" -d "$OUT/p2" -o run --output-format csv \
    -- python3 bench.py --steps 1 --warmup 0 --no-cpu ${BENCH_ARGS} > "$OUT/p2.log" 2>&1 || exit $?
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections, statistics
acc = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/p*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        acc[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(acc.items()):
    print(f"{k:32s} {c:24s} n={len(v):5d} median={statistics.median(v):14.1f}")
PY
