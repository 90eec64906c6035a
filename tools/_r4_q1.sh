#!/bin/bash
# one GPU call: full GPU tests on the in-tree build, then an interleaved A/B
# against a variant library:  tools/_r4_q1.sh <variant> [mode]
V=${1:?variant}; MODE=${2:-staged}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/q1_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/q1_tests.log; exit 1; }
tail -1 gpurun_out/q1_tests.log
timeout -k 10 500 bash tools/ab_libs.sh $MODE 2 base $V > gpurun_out/q1_ab.log 2>&1 || { tail -20 gpurun_out/q1_ab.log; exit 1; }
cat gpurun_out/q1_ab.log
