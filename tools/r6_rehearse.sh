#!/bin/bash
# The bench's N > 1 code path on a 1-GPU box: the plain line,
# the same at world 1 under torch.distributed.run (gloo group initialised),
# and two ranks sharing GPU 0 (--rehearse-on-gpu0).  Lines -> gpurun_out/rh_*.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
A=(--cpu-baseline 0 --host-rate 0 --variants 0)
timeout -k 10 200 python3 bench.py "${A[@]}" > gpurun_out/rh_plain.json 2> gpurun_out/rh_plain.err || exit 1
timeout -k 10 240 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 1 "${A[@]}" > gpurun_out/rh_world1.json 2> gpurun_out/rh_world1.err || exit 1
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29534 bench.py --gpus 2 --rehearse-on-gpu0 "${A[@]}" > gpurun_out/rh_world2.json 2> gpurun_out/rh_world2.err || exit 1
for f in plain world1 world2; do
  python3 -c "
import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], d['n_gpus'], d['value'], d['ms_per_step'], {k:v['ms'] for k,v in d['roofline']['kernels'].items()})" gpurun_out/rh_$f.json $f
done
