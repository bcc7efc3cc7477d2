#!/bin/bash
# SQ counters of the batch evaluation kernel, both forms (k_batch_top default,
# k_batch_eval with KSIM_BATCH_TILES=1), config 2: two PMC passes each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/${TAG:-pmc}
mkdir -p "$OUT"
run() {  # name, kernel regex, pass, counters...
  local name=$1 kre=$2 pass=$3; shift 3
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "$kre" -d "$OUT/$name/$pass" -o run \
    --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-adapt > "$OUT/$name.$pass.log" 2>&1
}
for v in top tiles; do
  unset KSIM_BATCH_TILES; kre=k_batch_top
  if [ $v = tiles ]; then export KSIM_BATCH_TILES=1; kre=k_batch_eval; fi
  run $v "$kre" p1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY || exit $?
  run $v "$kre" p2 SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_VALU_FP64 SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE || exit $?
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections, statistics
for v in ("top", "tiles"):
    acc = collections.defaultdict(list)
    for f in glob.glob(f"{sys.argv[1]}/{v}/p*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            acc[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), x in sorted(acc.items()):
        print(f"{v:6s} {k[:40]:40s} {c:22s} n={len(x):4d} median={statistics.median(x):14.1f}")
PY
