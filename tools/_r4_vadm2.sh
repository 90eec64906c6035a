#!/bin/bash
# one GPU call: all GPU tests, then the default bench interleaved with the
# HEAD library (3 rounds)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/vadm2_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/vadm2_tests.log; exit 1; }
tail -1 gpurun_out/vadm2_tests.log
timeout -k 10 600 bash tools/_r4_abenv.sh 3 head=FVAD_LIB=formula-vad_amd/lib/var/libfvad_head.so new=FVAD_X=1 \
  > gpurun_out/vadm2_ab.log 2>&1 || { tail -20 gpurun_out/vadm2_ab.log; exit 1; }
cut -c1-230 gpurun_out/vadm2_ab.log
