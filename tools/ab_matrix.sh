#!/bin/bash
# Bench a matrix of (library, environment) settings on the box, one short
# staged line each:  tools/ab_matrix.sh "<lib|base> <VAR=val|->" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
summ() { python3 -c "
import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d['value'], d['ms_per_step'], {k:v['ms'] for k,v in d['roofline']['kernels'].items()})" "$1" "$2"; }
i=0
for spec in "$@"; do
  set -- $spec
  lib=$1; sw=$2; i=$((i+1))
  L=""; [ "$lib" != base ] && L="FVAD_LIB=formula-vad_amd/lib/var/libfvad_$lib.so"
  E=""; [ "$sw" != - ] && E="$sw"
  env $L $E timeout -k 10 200 python3 bench.py --cpu-baseline 0 --host-rate 0 --variants 0 --resident-pushes 4 \
    > gpurun_out/abm_$i.log 2>&1 && summ gpurun_out/abm_$i.log "$lib $sw" || { tail -20 gpurun_out/abm_$i.log; exit 1; }
done
