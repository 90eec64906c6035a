#!/bin/bash
# one GPU call: k_plpcs parity (full-size, bit-exact) then A/B of its segment length
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_fp16.py -x -v --timeout 280 --timeout-method thread \
  -k "overlap" > gpurun_out/b_ovtest.log 2>&1 || { echo "overlap test failed"; tail -30 gpurun_out/b_ovtest.log; exit 1; }
tail -2 gpurun_out/b_ovtest.log
for rep in 1 2; do
  for OV in 1 0; do
    FVAD_FP16_OVERLAP=$OV timeout -k 10 200 python3 bench.py --cpu-baseline 0 --host-rate 0 --variants 0 --resident-pushes 4 \
      --mode fp16 > gpurun_out/b_ov.log 2>&1 || { tail -20 gpurun_out/b_ov.log; exit 1; }
    python3 -c "
import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('fp16 overlap', sys.argv[2], d['value'], d['ms_per_step'], {k:round(v['ms'],3) for k,v in d['roofline']['kernels'].items()})" gpurun_out/b_ov.log $OV
  done
done
FVAD_PLPC_K=4 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 \
  --timeout-method thread -k "not fp16" > gpurun_out/b_ps.log 2>&1 || { echo "plpcs tests failed"; tail -30 gpurun_out/b_ps.log; exit 1; }
tail -1 gpurun_out/b_ps.log
summ() { python3 -c "
import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k=d['roofline']['kernels'];print(sys.argv[2], d['value'], d['ms_per_step'], k['k_plpc']['ms'], k['k_pcorr']['ms'], k['k_fftAw']['ms'])" "$1" "$2"; }
for rep in 1 2; do
  for K in 0 4 8; do
    FVAD_PLPC_K=$K timeout -k 10 200 python3 bench.py --cpu-baseline 0 --host-rate 0 --variants 0 --resident-pushes 4 \
      > gpurun_out/b_psk.log 2>&1 && summ gpurun_out/b_psk.log "K=$K" || { tail -20 gpurun_out/b_psk.log; exit 1; }
  done
done
timeout -k 10 400 bash tools/ab_libs.sh staged 1 pr12 pr20 pr24u2 base > gpurun_out/b_pr.log 2>&1 || { tail -20 gpurun_out/b_pr.log; exit 1; }
cat gpurun_out/b_pr.log
