#!/bin/bash
# one GPU call: all GPU tests on the FD4 variant library with completed-wait
# skipping, then default-bench A/B rounds: in-tree build vs FD4 vs the skip
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
FVAD_LIB=$PWD/formula-vad_amd/lib/var/libfvad_fd4.so FVAD_WAIT_SKIP=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/fd4_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/fd4_tests.log; exit 1; }
tail -1 gpurun_out/fd4_tests.log
timeout -k 10 700 bash tools/_r4_abenv.sh 3 base=FVAD_X=1 fd4=FVAD_LIB=formula-vad_amd/lib/var/libfvad_fd4.so skip=FVAD_WAIT_SKIP=1 \
  > gpurun_out/fd4_ab.log 2>&1 || { tail -20 gpurun_out/fd4_ab.log; exit 1; }
cut -c1-230 gpurun_out/fd4_ab.log
