#!/bin/bash
# Round 3: config 1 scaled under ADAPT (the normalized-score pods on the ADAPT
# batch path), and config 2 / config 4 ADAPT, for every library variant in
# VARIANTS ("default" or a flavor tag), interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$PWD/gpurun_out/${TAG:-r03adc1}
mkdir -p "$OUT"
for v in ${VARIANTS:-default}; do
  lib=$v; [[ $v == default ]] && lib=""
  for c in ${CONFIGS:-1 2 4}; do
    case $c in
      1) args="--config 1 --mode adapt --steps 2 --warmup 1" ;;
      2) args="--mode adapt --no-adapt --steps 5 --warmup 2" ;;
      4) args="--config 4 --mode adapt --steps 2 --warmup 1" ;;
    esac
    KSIM_LIB_VARIANT=$lib timeout -k 10 300 python3 -u bench.py $args --no-cpu > "$OUT/c${c}a_$v.json" 2> "$OUT/c${c}a_$v.err" || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1].split('/')[-1], '%.3f ms' % d['ms_per_step'], d['batch_stats'], {n: round(v['avg_ms'] * 1e3, 2) for n, v in d['kernels'].items() if not n.startswith('_')})" "$OUT/c${c}a_$v.json"
  done
done
