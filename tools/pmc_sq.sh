#!/bin/bash
# SQ counter passes (issue / wait / LDS behaviour per kernel) of the default
# bench workload; each pass is its own rocprofv3 run (no other trace domain).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/sq_${1:-run}
mkdir -p "$OUT"
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_INSTS_FLAT SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM"; do
  timeout -k 10 300 rocprofv3 --pmc $set -d "$OUT/p$i" -o run -- python3 bench.py --cpu-baseline 0 --host-rate 0 --variants 0 --steps 2 --warmup 1 \
    > "$OUT/p$i.log" 2>&1
  i=$((i+1))
done
