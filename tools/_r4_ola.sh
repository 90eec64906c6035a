#!/bin/bash
# one GPU call: the tests that cover k_olafb (parity, full size, streaming,
# config, vadm, simulator), then base vs a variant A/B:  tools/_r4_ola.sh <variant>
V=${1:?variant}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/ola_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/ola_tests.log; exit 1; }
tail -1 gpurun_out/ola_tests.log
timeout -k 10 500 bash tools/ab_libs.sh staged 2 base $V > gpurun_out/ola_ab.log 2>&1 || { tail -20 gpurun_out/ola_ab.log; exit 1; }
cat gpurun_out/ola_ab.log
