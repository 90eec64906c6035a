#!/bin/bash
# Quick GPU check on the box: the staged / fused parity tests, the full-size
# bench-configuration parity test, then a short bench line per mode.
#   tools/quick.sh [pytest -k expression]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
K=${1:-"test_engine_bit_exact_ragged or test_engine_channels or test_configs3_shard or test_fp16_ragged"}
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$K" \
  > gpurun_out/quick_test.log 2>&1 || { tail -30 gpurun_out/quick_test.log; exit 1; }
tail -1 gpurun_out/quick_test.log
summ() { python3 -c "
import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d['value'], d['ms_per_step'], {k:v['ms'] for k,v in d['roofline']['kernels'].items()})" "$1" "$2"; }
for m in staged fp16; do
  timeout -k 10 200 python3 bench.py --cpu-baseline 0 --host-rate 0 --mode $m > gpurun_out/quick_$m.log 2>&1 \
    && summ gpurun_out/quick_$m.log $m || { tail -20 gpurun_out/quick_$m.log; exit 1; }
done
