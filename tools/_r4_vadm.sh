#!/bin/bash
# one GPU call: all GPU tests on the in-tree build, then an env A/B
# (staged and fp16, twice each):  tools/_r4_vadm.sh VAR=value
SW=${1:?VAR=value}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/vadm_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/vadm_tests.log; exit 1; }
tail -1 gpurun_out/vadm_tests.log
timeout -k 10 700 bash tools/ab_quick.sh "$SW" > gpurun_out/vadm_ab.log 2>&1 || { tail -20 gpurun_out/vadm_ab.log; exit 1; }
cat gpurun_out/vadm_ab.log
