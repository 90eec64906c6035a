#!/bin/bash
# Kernel-trace + PMC traffic profile of the default bench workload, run on the
# GPU box:  tools/profile.sh <tag> [bench args...]
# Three separate rocprofv3 passes (trace/stats, FETCH_SIZE, WRITE_SIZE; PMC
# passes never combined with other trace domains), then tools/pmc_summary.py
# writes profiles/<tag>_kernel_stats.csv and profiles/pmc_traffic.json.
set -euo pipefail
TAG=${1:?tag}
shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
BENCH=(bench.py --cpu-baseline 0 --host-rate 0 --variants 0 --one-engine-leg 0 "$@")
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run -- python3 "${BENCH[@]}" --steps 20 --warmup 10 \
  > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run -- python3 "${BENCH[@]}" --steps 2 --warmup 1 \
  > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run -- python3 "${BENCH[@]}" --steps 2 --warmup 1 \
  > "$OUT/write.log" 2>&1
python3 tools/pmc_summary.py "$OUT" "$TAG" "$@"
