#!/bin/bash
# GPU check: the named test files (default: parity + streaming), then a
# bench line with its kernel table and host-fed rates.
#   tools/r6_check.sh <tag> [test files...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:?tag}
shift
mkdir -p gpurun_out
T=("$@")
[ ${#T[@]} -eq 0 ] && T=(tests/test_gpu_parity.py tests/test_gpu_streaming.py)
timeout -k 10 600 python3 -u -m pytest "${T[@]}" -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python3 bench.py --cpu-baseline 0 --variants 0 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
  || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python3 - gpurun_out/${TAG}_bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
h = d.get("host_buffers") or {}
print("value %.4g ms %.3f host %s i16 %s pageable %s" % (d["value"], d["ms_per_step"], h.get("ms_per_step"),
      h.get("i16_ms_per_step"), h.get("pageable_ms_per_step")))
print({k: v["ms"] for k, v in d["roofline"]["kernels"].items()})
PY
