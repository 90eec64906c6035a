#!/bin/bash
# one GPU call: k_pcorr LDS / VALU counters of the in-tree build and of the
# diagnostic builds without Q1 (skip1), Q3 (skip2) or Q5's (skip4) sums --
# the per-phase attribution of VERDICT r3 #3 -- plus their k_pcorr times
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
for L in base skip1 skip2 skip4; do
  if [ "$L" == base ]; then LIBP=$PWD/formula-vad_amd/lib/libfvad.so; else LIBP=$PWD/formula-vad_amd/lib/var/libfvad_$L.so; fi
  FVAD_LIB=$LIBP timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU \
    -d gpurun_out/lds_$L -o run -- python3 bench.py --cpu-baseline 0 --host-rate 0 --variants 0 --steps 2 --warmup 1 \
    > gpurun_out/lds_$L.log 2>&1 || { echo "pmc $L failed"; tail -20 gpurun_out/lds_$L.log; exit 1; }
  echo "== $L"; python3 tools/sq_summary.py gpurun_out/lds_$L k_pcorr
  FVAD_LIB=$LIBP timeout -k 10 200 python3 bench.py --cpu-baseline 0 --host-rate 0 --variants 0 --resident-pushes 4 \
    > gpurun_out/ldst_$L.log 2>&1 || { tail -20 gpurun_out/ldst_$L.log; exit 1; }
  python3 -c "
import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('  k_pcorr ms', d['roofline']['kernels']['k_pcorr']['ms'])" gpurun_out/ldst_$L.log
done
