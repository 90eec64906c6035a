#!/bin/bash
# Interleaved A/B of library builds (tools/variant.sh) with short bench runs:
#   tools/ab_libs.sh "<mode>" <reps> <name|base>... [-- bench args]
# Each name is formula-vad_amd/lib/var/libfvad_<name>.so; "base" is the
# in-tree build.  One summary line per run: value, ms/push, kernel ms.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
MODE=$1; REPS=$2; shift 2
LIBS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do LIBS+=("$1"); shift; done
[ "$1" == "--" ] && shift
summ() { python3 -c "
import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d['value']/1e6,2), d['ms_per_step'], {k:round(v['ms'],3) for k,v in d['roofline']['kernels'].items()})" "$1" "$2"; }
for rep in $(seq "$REPS"); do
  for L in "${LIBS[@]}"; do
    if [ "$L" == base ]; then LIBP=formula-vad_amd/lib/libfvad.so; else LIBP=formula-vad_amd/lib/var/libfvad_$L.so; fi
    FVAD_LIB=$LIBP timeout -k 10 200 python3 bench.py --cpu-baseline 0 --host-rate 0 --variants 0 --resident-pushes 4 \
      --mode "$MODE" "$@" > gpurun_out/abl_$L.log 2>&1 && summ gpurun_out/abl_$L.log "$MODE $L" || { tail -20 gpurun_out/abl_$L.log; exit 1; }
  done
done
