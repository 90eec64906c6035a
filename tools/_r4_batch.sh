#!/bin/bash
# one GPU call: x_lp rows from k_prep3 (parity), then A/B of the k_fftAw fork
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_streaming.py -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/b_xlp.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/b_xlp.log; exit 1; }
tail -1 gpurun_out/b_xlp.log
FVAD_FORK=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -x -q --timeout 280 --timeout-method thread \
  -k "staged_every_stream or fp16" > gpurun_out/b_fork.log 2>&1 || { echo "fork tests failed"; tail -30 gpurun_out/b_fork.log; exit 1; }
tail -1 gpurun_out/b_fork.log
timeout -k 10 700 bash tools/ab_quick.sh FVAD_FORK=1 > gpurun_out/b_abf.log 2>&1 || { tail -20 gpurun_out/b_abf.log; exit 1; }
cat gpurun_out/b_abf.log
