#!/bin/bash
# one GPU call: full GPU test suite + smoke, the default bench line, and the
# rocprof kernel-trace / PMC profiles of both modes:  tools/_r4_base.sh <tag>
TAG=${1:?tag}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/base_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/base_tests.log; exit 1; }
tail -1 gpurun_out/base_tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/base_smoke.log 2>&1 \
  || { tail -20 gpurun_out/base_smoke.log; exit 1; }
tail -1 gpurun_out/base_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/base_bench.log 2>&1 || { tail -20 gpurun_out/base_bench.log; exit 1; }
tail -1 gpurun_out/base_bench.log > gpurun_out/${TAG}_staged_bench.json
timeout -k 10 900 bash tools/profile.sh ${TAG}_staged > gpurun_out/base_prof_s.log 2>&1 || { tail -20 gpurun_out/base_prof_s.log; exit 1; }
timeout -k 10 900 bash tools/profile.sh ${TAG}_fp16 --mode fp16 > gpurun_out/base_prof_f.log 2>&1 || { tail -20 gpurun_out/base_prof_f.log; exit 1; }
cp profiles/pmc_traffic*.json gpurun_out/ 2>/dev/null
ls profiles | grep "$TAG" | sed 's/^/profiles\//' | xargs -I{} cp {} gpurun_out/

# stream-count scaling of the per-kernel times (rounds vs throughput)
for B in 1536 1024; do
  timeout -k 10 200 python3 bench.py --cpu-baseline 0 --host-rate 0 --variants 0 --resident-pushes 4 --streams-per-gpu $B \
    > gpurun_out/base_scale_$B.log 2>&1 || break
  python3 -c "
import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d['value']/1e6,2), d['ms_per_step'], {k:round(v['ms'],3) for k,v in d['roofline']['kernels'].items()})" gpurun_out/base_scale_$B.log $B
done
echo done
