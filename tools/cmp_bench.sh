#!/bin/bash
# Bench the default library and every variant in formula-vad_amd/lib/var on
# the GPU box (one line each: name, value, ms/step, per-kernel ms).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
summ() { python3 -c "
import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d['value'], d['ms_per_step'], {k:v['ms'] for k,v in d['roofline']['kernels'].items()})" "$1" "$2"; }
timeout -k 10 200 python3 bench.py --cpu-baseline 0 "$@" > gpurun_out/cmp_base.log 2>&1 && summ gpurun_out/cmp_base.log base
for f in $(ls formula-vad_amd/lib/var/*.so 2>/dev/null); do
  n=$(basename "$f" .so)
  FVAD_LIB=$f timeout -k 10 200 python3 bench.py --cpu-baseline 0 "$@" > gpurun_out/cmp_$n.log 2>&1 && summ gpurun_out/cmp_$n.log $n || exit 1
done
