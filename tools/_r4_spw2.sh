#!/bin/bash
# k_gru16 with 8 streams per workgroup by default: the fp16 tests (overlap
# mode included, on 16) and the fp16 full-size tolerance test, then fp16 bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fp16.py tests/test_gpu_fullsize.py -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/spw2_tests.log 2>&1 || { tail -30 gpurun_out/spw2_tests.log; exit 1; }
tail -1 gpurun_out/spw2_tests.log
bash tools/ab_libs.sh fp16 2 base
