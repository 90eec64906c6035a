#!/bin/bash
# k_gru16 streams per workgroup (FVAD_GRU_SPW=8 variant): fp16 parity tests on
# the variant, then interleaved fp16 bench A/B against the in-tree build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
FVAD_LIB=$PWD/formula-vad_amd/lib/var/libfvad_spw8.so timeout -k 10 400 python -u -m pytest tests/test_gpu_fp16.py -x -q -k "not overlap" \
  --timeout 200 --timeout-method thread > gpurun_out/spw_tests.log 2>&1 || { tail -30 gpurun_out/spw_tests.log; exit 1; }
tail -1 gpurun_out/spw_tests.log
bash tools/ab_libs.sh fp16 3 base spw8
