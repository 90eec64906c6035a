#!/bin/bash
# one GPU call: fp16 overlap identity test first (its own time limit), then
# the A/B measurements; every step bounded, the chain stops at the first failure
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_fp16.py -x -v --timeout 280 --timeout-method thread \
  -k "overlap" > gpurun_out/b_ovtest.log 2>&1 || { echo "overlap test failed"; tail -30 gpurun_out/b_ovtest.log; exit 1; }
tail -2 gpurun_out/b_ovtest.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_fp16.py tests/test_gpu_vadm.py -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/b_fp16.log 2>&1 || { echo "fp16 tests failed"; tail -30 gpurun_out/b_fp16.log; exit 1; }
tail -1 gpurun_out/b_fp16.log
timeout -k 10 600 bash tools/ab_quick.sh FVAD_FP16_OVERLAP=0 > gpurun_out/b_abov.log 2>&1 || { tail -20 gpurun_out/b_abov.log; exit 1; }
cat gpurun_out/b_abov.log
timeout -k 10 250 python -u tools/split_probe.py staged 12 > gpurun_out/b_split.log 2>&1 || { tail -20 gpurun_out/b_split.log; exit 1; }
cat gpurun_out/b_split.log
timeout -k 10 300 bash tools/ab_libs.sh staged 2 base lt8 lt32 > gpurun_out/b_ablt.log 2>&1 || { tail -20 gpurun_out/b_ablt.log; exit 1; }
cat gpurun_out/b_ablt.log
