#!/bin/bash
# Round 3: the deferred-commit P100 batches -- parity tests, then config 2
# default (deferred commit) against KSIM_NO_LAZY=1 (three launches), same box,
# and the rocprof kernel stats of the default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/${TAG:-r03lazy}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_ab_switches.py} -x -v --timeout 240 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; if [ $rc -ne 0 ]; then exit $rc; fi
for r in 1 2; do
  for v in lazy nolazy; do
    if [ $v == nolazy ]; then export KSIM_NO_LAZY=1; else unset KSIM_NO_LAZY; fi
    timeout -k 10 200 python3 -u bench.py --steps 5 --warmup 2 --no-cpu > "$OUT/c2_${v}_$r.json" 2> "$OUT/c2_${v}_$r.err" || exit $?
  done
done
unset KSIM_NO_LAZY
python3 - "$OUT" <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/c2_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    k = d["kernels"]
    print(f.split("/")[-1], "%.3f ms" % d["ms_per_step"], "adapt %.3f ms" % d["adapt"]["ms_per_step"], d["batch_stats"],
          {n: round(v["avg_ms"] * 1e3, 2) for n, v in k.items() if not n.startswith("_")}, d["roofline"]["kernel"], round(d["roofline"]["avg_launch_ms"] * 1e3, 2))
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv -- \
  python3 -u bench.py --no-cpu --no-adapt > "$OUT/bench_stats.json" 2> "$OUT/bench_stats.err" || exit $?
find "$OUT/stats" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
cut -c1-60,200- "$OUT/kernel_stats.csv" | head -6
