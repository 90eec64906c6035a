#!/bin/bash
# End-of-round evidence on one MI355X: the whole GPU suite, smoke(), the
# default bench line and its wall time (the rocprofv3 kernel-trace + PMC profile: tools/profile.sh <tag>,
# in a call of its own).
#   tools/r6_final.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:?tag}
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -s \
  > gpurun_out/${TAG}_gputests.log 2>&1 || { tail -40 gpurun_out/${TAG}_gputests.log; exit 1; }
tail -1 gpurun_out/${TAG}_gputests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 \
  || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
t0=$(date +%s)
timeout -k 10 400 python3 bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
  || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
echo "bench wall time $(( $(date +%s) - t0 )) s"
python3 - gpurun_out/${TAG}_bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value %.5g ms %.3f frac %s" % (d["value"], d["ms_per_step"], d["roofline"]["frac"]))
PY
