#!/bin/bash
# one GPU call: kernel-trace runs of the default bench for several env
# settings (rocprofv3 --kernel-trace only):  tools/_r4_trace.sh NAME=ENV ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
for spec in "$@"; do
  name=${spec%%=*}; envs=${spec#*=}
  env $envs timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tr_$name -o run -- python3 bench.py --cpu-baseline 0 \
    --host-rate 0 --variants 0 --steps 20 --warmup 10 > gpurun_out/tr_$name.log 2>&1 || { tail -20 gpurun_out/tr_$name.log; exit 1; }
  tail -1 gpurun_out/tr_$name.log | cut -c1-200
done
