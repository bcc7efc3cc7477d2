#!/bin/bash
# Counter passes over the batch kernels (one rocprofv3 run per pass; no trace domains).
set -e
cd /tmp && export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc
mkdir -p $OUT
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
P2="SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU SQ_INSTS_MFMA"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex "k_batch" -d $OUT/p$i -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/prof_batch.py 1280 > $OUT/p$i.log 2>&1
done
