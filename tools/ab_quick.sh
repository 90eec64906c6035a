#!/bin/bash
# A/B an environment switch with short bench runs (staged, then fp16), each
# side twice, interleaved:  tools/ab_quick.sh VAR=value [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
SW=$1; shift
summ() { python3 -c "
import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d['value'], d['ms_per_step'], {k:v['ms'] for k,v in d['roofline']['kernels'].items()})" "$1" "$2"; }
for m in staged fp16; do
  for rep in 1 2; do
    timeout -k 10 200 python3 bench.py --cpu-baseline 0 --host-rate 0 --variants 0 --resident-pushes 4 --mode $m "$@" \
      > gpurun_out/abq_base.log 2>&1 && summ gpurun_out/abq_base.log "$m base" || { tail -20 gpurun_out/abq_base.log; exit 1; }
    env "$SW" timeout -k 10 200 python3 bench.py --cpu-baseline 0 --host-rate 0 --variants 0 --resident-pushes 4 --mode $m "$@" \
      > gpurun_out/abq_sw.log 2>&1 && summ gpurun_out/abq_sw.log "$m $SW" || { tail -20 gpurun_out/abq_sw.log; exit 1; }
  done
done
