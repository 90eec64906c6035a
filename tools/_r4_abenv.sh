#!/bin/bash
# one GPU call: the default bench line (staged) for several env settings,
# interleaved, REPS rounds:  tools/_r4_abenv.sh REPS NAME=ENV ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
REPS=$1; shift
summ() { python3 -c "
import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d['value']/1e6,3), d['ms_per_step'], {k:round(v['ms'],3) for k,v in d['roofline']['kernels'].items()})" "$1" "$2"; }
for rep in $(seq "$REPS"); do
  for spec in "$@"; do
    name=${spec%%=*}; envs=${spec#*=}
    env $envs timeout -k 10 200 python3 bench.py --cpu-baseline 0 --host-rate 0 --variants 0 > gpurun_out/abe_$name.log 2>&1 \
      && summ gpurun_out/abe_$name.log "$name" || { tail -20 gpurun_out/abe_$name.log; exit 1; }
  done
done
