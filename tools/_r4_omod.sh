#!/bin/bash
# one GPU call: the parity / full-size / streaming tests on the
# FVAD_PREP_OMOD=1 variant, then default-bench A/B rounds against the in-tree build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
FVAD_LIB=$PWD/formula-vad_amd/lib/var/libfvad_omod.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py \
  tests/test_gpu_fullsize.py tests/test_gpu_streaming.py tests/test_gpu_config.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/omod_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/omod_tests.log; exit 1; }
tail -1 gpurun_out/omod_tests.log
timeout -k 10 700 bash tools/_r4_abenv.sh 3 base=FVAD_X=1 omod=FVAD_LIB=$PWD/formula-vad_amd/lib/var/libfvad_omod.so \
  > gpurun_out/omod_ab.log 2>&1 || { tail -20 gpurun_out/omod_ab.log; exit 1; }
cut -c1-200 gpurun_out/omod_ab.log
