#!/bin/bash
# one GPU call: parity tests of the in-tree build, stamps of the in-tree and
# old-Q1 stamp builds, A/B of base vs q1old
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/q1b_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/q1b_tests.log; exit 1; }
tail -1 gpurun_out/q1b_tests.log
FVAD_LIB=formula-vad_amd/lib/libfvad_stamps.so timeout -k 10 120 python -u tools/stamps.py 2048 50 staged > gpurun_out/q1b_stamps_new.log 2>&1 || { tail -20 gpurun_out/q1b_stamps_new.log; exit 1; }
FVAD_LIB=formula-vad_amd/lib/var/libfvad_st0.so timeout -k 10 120 python -u tools/stamps.py 2048 50 staged > gpurun_out/q1b_stamps_old.log 2>&1 || { tail -20 gpurun_out/q1b_stamps_old.log; exit 1; }
grep -A8 "k_pcorr" gpurun_out/q1b_stamps_new.log gpurun_out/q1b_stamps_old.log
timeout -k 10 500 bash tools/ab_libs.sh staged 2 base q1old > gpurun_out/q1b_ab.log 2>&1 || { tail -20 gpurun_out/q1b_ab.log; exit 1; }
cat gpurun_out/q1b_ab.log
