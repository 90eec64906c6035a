"""world_size-2 gloo run of bench.py's multi-GPU logic on CPU: rendezvous on
127.0.0.1, disjoint stream partitions per rank, barrier, max-over-ranks timing
and the whole-job rate (the N>1 path the driver launches with
torch.distributed.run, minus the GPU).  bench.py's process group is gloo at
every N (CPU tensors, no RCCL), so this is the production collective path."""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    sys.path.insert(0, ROOT)
    import bench
    r, w, local, dist, torch = bench.dist_setup(world)
    assert dist.get_backend() == "gloo"  # the production path: no RCCL at any N
    base, n = bench.stream_partition(r, 2048)
    bench.barrier(dist, torch)
    elapsed = 1.0 + r  # rank 1 is the slow one
    mx = bench.max_over_ranks(elapsed, dist, torch)
    assert not torch.cuda.is_initialized()  # barrier / max-reduce touch no HIP stream
    ids = torch.tensor([base, base + n], dtype=torch.int64)
    gathered = [torch.zeros(2, dtype=torch.int64) for _ in range(w)]
    dist.all_gather(gathered, ids)
    q.put((r, w, mx, [g.tolist() for g in gathered], bench.aggregate_rate(2048 * 2 * 50, w, 10, mx)))
    dist.destroy_process_group()


def test_two_rank_partition_and_timing():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for r, w, mx, parts, rate in res:
        assert w == 2 and mx == 2.0
        assert parts == [[0, 2048], [2048, 4096]]  # disjoint, contiguous stream ids
        assert rate == pytest.approx(2048 * 2 * 50 * 2 * 10 / 2.0)


def test_bench_self_launch_two_ranks():
    """`bench.py --gpus 2` outside torch.distributed.run re-launches itself as
    two ranks (child torch.distributed.run on 127.0.0.1); --cpu-stub swaps the
    engine for a CPU stub so the launcher, partition, barrier and max-reduce
    run here on gloo.  Rank 1 sleeps longer: the reported time is the max."""
    import json
    import subprocess
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--cpu-stub",
                          "--steps", "4", "--warmup", "1"], capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1  # one JSON line, from rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2
    assert d["ms_per_step"] >= 20.0  # rank 1's 20 ms per step, not rank 0's 10
    assert d["value"] == pytest.approx(2048 * 2 * 50 * 2 / (d["ms_per_step"] / 1000.0), rel=1e-6)
    # per-rank kernel tables, max over ranks per kernel (the slowest rank sets the step)
    ro = d["roofline"]
    assert ro["kernels"] == {"k_a": 2.0, "k_b": 2.0}
    assert ro["ranks"]["max_rank"] == {"k_a": 1, "k_b": 0}
    assert set(ro["ranks"]["per_rank"]) == {"0", "1"}


def test_bench_has_no_rccl_path():
    """The bench's collectives are gloo only: no RCCL
    communicator or torch HIP stream beside the engine's streams."""
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert "nccl" not in src and "torch.cuda" not in src


def test_bench_world_one_under_launcher():
    """--gpus 1 under torch.distributed.run (world 1): the gloo group is
    initialised like at N > 1 and the line carries the per-rank table."""
    import json
    import subprocess
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                          "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
                          os.path.join(ROOT, "bench.py"), "--gpus", "1", "--cpu-stub", "--steps", "3", "--warmup", "1"],
                         capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and set(d["roofline"]["ranks"]["per_rank"]) == {"0"}
