#!/bin/bash
# A/B an environment switch on the box: bench lines with and without it.
#   tools/ab_env.sh VAR=value [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
SW=$1; shift
summ() { python3 -c "
import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d['value'], d['ms_per_step'], {k:v['ms'] for k,v in d['roofline']['kernels'].items()})" "$1" "$2"; }
for m in staged fp16; do
  timeout -k 10 200 python3 bench.py --cpu-baseline 0 --host-rate 0 --mode $m "$@" > gpurun_out/ab_base_$m.log 2>&1 \
    && summ gpurun_out/ab_base_$m.log "$m base" || { tail -20 gpurun_out/ab_base_$m.log; exit 1; }
  env "$SW" timeout -k 10 200 python3 bench.py --cpu-baseline 0 --host-rate 0 --mode $m "$@" > gpurun_out/ab_sw_$m.log 2>&1 \
    && summ gpurun_out/ab_sw_$m.log "$m $SW" || { tail -20 gpurun_out/ab_sw_$m.log; exit 1; }
done
