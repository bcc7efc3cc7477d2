#!/bin/bash
# Extra bench lines on one GPU: config 3 (topology), forced sharded path (1-rank RCCL), config 2 ADAPT.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/${TAG:-run}
mkdir -p "$OUT"
step() { echo "== $*" >&2 ; "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step timeout -k 10 300 python -u bench.py --config 3 --steps 1 --warmup 1 --cpu-seconds 10 > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err"
step timeout -k 10 200 python -u bench.py --force-shard --no-cpu > "$OUT/bench_shard1.json" 2> "$OUT/bench_shard1.err"
step timeout -k 10 200 python -u bench.py --mode adapt --steps 1 --warmup 1 --cpu-seconds 10 > "$OUT/bench_adapt.json" 2> "$OUT/bench_adapt.err"
echo done
