#!/bin/bash
# One GPU call: k_pcorr's LDS / VALU counters (rocprofv3 --pmc, default bench,
# 2 steps) and k_pcorr event times (bench, 4 resident pushes) of the in-tree
# build and of the diagnostic flavours `make -C formula-vad_amd diag DIAG=<bits>`
# (built beforehand on the CPU): FVAD_DIAG_SKIP 1 / 2 / 4 drop Q1's / Q3's /
# Q5's sums (per-phase attribution), 8 reads Q1's y operands at a
# conflict-free lane stride (wrong values: the upper bound of a conflict-free
# Q1 layout).  Usage: tools/lds_attr.sh base 8 1 ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
for L in "$@"; do
  if [ "$L" == base ]; then LIBP=$PWD/formula-vad_amd/lib/libfvad.so; else LIBP=$PWD/formula-vad_amd/lib/libfvad_diag$L.so; fi
  FVAD_LIB=$LIBP timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU \
    -d gpurun_out/lds_$L -o run -- python3 bench.py --cpu-baseline 0 --host-rate 0 --variants 0 --steps 2 --warmup 1 \
    > gpurun_out/lds_$L.log 2>&1 || { echo "pmc $L failed"; tail -20 gpurun_out/lds_$L.log; exit 1; }
  echo "== $L"; python3 tools/sq_summary.py gpurun_out/lds_$L k_pcorr
  FVAD_LIB=$LIBP timeout -k 10 200 python3 bench.py --cpu-baseline 0 --host-rate 0 --variants 0 --resident-pushes 4 \
    > gpurun_out/ldst_$L.log 2>&1 || { tail -20 gpurun_out/ldst_$L.log; exit 1; }
  python3 -c "
import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('  k_pcorr ms', d['roofline']['kernels']['k_pcorr']['ms'])" gpurun_out/ldst_$L.log
done
