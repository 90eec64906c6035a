#!/usr/bin/env python3
"""Bench: Formula-VAD per-frame hot path on MI355X.

Metric (BASELINE.json): 48 kHz 480-sample VAD frames/sec whole node; max
concurrent real-time streams.  A VAD frame = one 480-sample channel-frame
through rnnoise (+ its share of the 2048-point band-energy FFT).

Workload: configs[4]'s per-GPU partition — 2048 synthetic 48 kHz stereo
streams per GPU (16384 at 8 GPUs), weak scaling, f32 exact numerics.  A step
= one push of TICKS ticks (480 samples per channel) for every stream of the
partition — the staged pipeline's kernels (fvad_staged.hip; --mode fused:
k_prep + k_frame) on the engine's HIP streams, input resident in HBM, device
VADMachine included.

Multi-GPU: one process per GPU.  Under torch.distributed.run (WORLD_SIZE set)
each rank runs its own stream partition; `--gpus N` without WORLD_SIZE
re-launches this script under torch.distributed.run with N ranks as a child
process, before anything touches the GPU.  The only collectives are the
barrier and the max-reduce of the timing (no data-path collective).

Also reported (never `value`): host_buffers, the streaming rate with the
input coming from host memory each push (fvad_engine_submit: pinned slots,
H2D overlapped with the previous push), and cpu_baseline, the oracle's whole
per-stream path on this host's cores.

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "formula-vad_amd"))

METRIC = "48 kHz 480-sample VAD frames/sec whole node; max concurrent real-time streams"
HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP32_PEAK_TFLOPS = 157.3    # MI355X_MICROARCH.md: FP32 vector peak (FMA = 2 flops per lane per cycle)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # a timed region starts with no push in flight, so its first push runs its
    # k_prep3 (~3 ms) unoverlapped; 30 steps keep that fill under 2 % of the
    # steady-state streaming rate (10 steps: ~5 %)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--streams-per-gpu", type=int, default=2048)
    ap.add_argument("--channels", type=int, default=2)
    ap.add_argument("--ticks", type=int, default=50)
    ap.add_argument("--mode", choices=("staged", "fused", "fp16"), default="staged",
                    help="staged (bit-exact, default), fused (bit-exact), fp16 (configs[4]: GRU on MFMA, tolerance)")
    ap.add_argument("--no-vadm", action="store_true", help="staged: do not run the device VADMachine (k_vadm)")
    ap.add_argument("--cpu-baseline", type=int, default=1, help="time the CPU oracle on this host (rank 0)")
    ap.add_argument("--cpu-streams", type=int, default=64)
    ap.add_argument("--cpu-ticks", type=int, default=100)
    ap.add_argument("--cpu-seconds", type=float, default=8.0,
                    help="measure each CPU sample (single-core, all-core) for about this long")
    ap.add_argument("--pmc-json", default=None,
                    help="PMC byte counts (tools/profile.sh); default profiles/pmc_traffic[_<mode>].json")
    ap.add_argument("--host-rate", type=int, default=1,
                    help="also time pushes from host buffers (PCIe-inclusive; reported as host_buffers, never value)")
    ap.add_argument("--cpu-stub", action="store_true",
                    help="no GPU: gloo ranks with a stub engine (tests the launcher, barrier and max-reduce)")
    ap.add_argument("--variants", type=int, default=1,
                    help="staged runs: also time the fp16 engine mode (configs[4]'s variant) on the same "
                         "workload and report it under `variants` (never `value`)")
    return ap.parse_args()


def maybe_spawn(args):
    """`--gpus N` (N > 1) outside torch.distributed.run: start N ranks as a
    child torch.distributed.run (one process per GPU) and exit with its code.
    Runs before anything touches the GPU, so no process that initialised HIP
    is replaced."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    sys.exit(subprocess.call(cmd, env=env))


def dist_setup(n_gpus, backend="nccl"):
    """One process per GPU (torch.distributed.run env).  backend "gloo" is
    used by the CPU tests of this logic (tests/test_dist_cpu.py).  Under
    torch.distributed.run the world size is the launcher's; it must match
    --gpus when that was given explicitly."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if n_gpus > 1 and world != n_gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d" % (n_gpus, world))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        return rank, world, local, dist, torch
    return rank, world, local, None, None


def _on_gpu(dist):
    return dist.get_backend() == "nccl"


def barrier(dist, torch):
    if dist is not None:
        dist.barrier()
        if _on_gpu(dist):
            torch.cuda.synchronize()


def max_over_ranks(x, dist, torch):
    if dist is None:
        return x
    t = torch.tensor([x], dtype=torch.float64, device="cuda" if _on_gpu(dist) else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def stream_partition(rank, streams_per_gpu):
    """Weak scaling: rank r owns synthetic stream ids [r*B, (r+1)*B) (configs[3]/[4]);
    streams are independent, so there is no data-path collective."""
    return rank * streams_per_gpu, streams_per_gpu


def aggregate_rate(frames_per_rank_step, world, steps, elapsed_max):
    """Whole-job channel-frames/s: every rank's frames over the slowest rank's time."""
    return frames_per_rank_step * world * steps / elapsed_max


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            return next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), "")
    except OSError:
        return ""


def cpu_baseline(args):
    """The oracle's whole per-stream path (rnnoise + re-block + FFT B band sums
    + VADMachine: ora_bench_pipeline, the same work scope as the GPU step),
    built -O3 -march=native -ffp-contract=off on this host, run single-core
    and on the cores this process may use (at most 16: the GPU box's share of
    its host).  Bounded sample: the first ticks of the same synthetic streams,
    pushed in 50-tick chunks like the GPU step, repeated for about
    --cpu-seconds each."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import oracle
    import fvad
    L, cpu_model = oracle.native_lib()
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    threads = max(1, min(16, avail))
    S, T, Ch = args.cpu_streams, args.cpu_ticks, args.channels
    n = T * 480
    pcm = np.zeros((S, Ch, n), np.float32)
    for s in range(S):
        pcm[s] = fvad.synth_stream(s * max(1, args.streams_per_gpu // S), n, Ch)[0]

    def timed(nthr, streams):
        secs, reps = 0.0, 0
        while secs < args.cpu_seconds and reps < 200:
            dt, _ = oracle.bench_pipeline(pcm[:streams], chunk=args.ticks * 480, n_threads=nthr, L=L)
            secs += dt
            reps += 1
        return streams * T * Ch * reps / secs, secs, reps

    one, one_s, one_r = timed(1, max(1, S // 16))
    allc, all_s, all_r = timed(threads, S)
    return {"value": round(allc, 1), "unit": "frames/s", "cores": threads, "kind": "port",
            "single_core": round(one, 1),
            "sample": "oracle whole path (rnnoise, FFT B band sums, VADMachine), -O3 -march=native "
                      "-ffp-contract=off on %s (nproc %s, %d usable); all-core: %d streams x %d ticks x %d ch, "
                      "%d threads, %d passes, %.1f s; single-core: %d streams, %d passes, %.1f s" % (
                          cpu_model, os.cpu_count(), avail, S, T, Ch, threads, all_r, all_s,
                          max(1, S // 16), one_r, one_s)}


class StubEngine:
    """--cpu-stub: stands in for fvad.Engine on a CPU-only gloo rank (tests
    the launcher, partition, barrier and max-reduce without a GPU)."""

    def __init__(self, n):
        self.n, self.runs = n, 0

    def run_resident(self, n_ticks):
        self.runs += 1

    def sync(self):
        pass


def stub_main(args):
    rank, world, local, dist, torch = dist_setup(args.gpus, backend="gloo")
    B, Ch, T = args.streams_per_gpu, args.channels, args.ticks
    base, _ = stream_partition(rank, B)
    eng = StubEngine(B)
    for _ in range(args.warmup):
        eng.run_resident(T)
    barrier(dist, torch)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.run_resident(T)
        time.sleep(0.01 * (1 + rank))
    barrier(dist, torch)
    elapsed = max_over_ranks(time.perf_counter() - t0, dist, torch)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": aggregate_rate(B * Ch * T, world, args.steps, elapsed),
                          "unit": "frames/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": 1000.0 * elapsed / args.steps, "data": "stub (no GPU)",
                          "config": {"streams_per_gpu": B, "first_stream": base}}), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def host_rate(eng, args, rank, dist, torch):
    """Streaming from host memory (fvad_engine_input_slot / submit / collect):
    two pushes in flight, the input's H2D copy over PCIe overlapping the
    previous push's kernels, outputs copied back every push.  pinned: the
    producer writes each push into the engine's pinned slot (the copy cost of
    the producer itself is not counted); pageable: submit from an ordinary
    host array (plus a threaded copy into the slot)."""
    import numpy as np
    B, Ch, T = args.streams_per_gpu, args.channels, args.ticks
    rng = np.random.default_rng(rank)
    src = (rng.standard_normal((T, B, Ch, 480), dtype=np.float32) * np.float32(0.05))
    res = {}
    for kind in ("pinned", "pageable"):
        if kind == "pinned":
            for _ in range(2):  # both slots hold a push's worth of input
                sl = eng.input_slot()
                sl[:T] = src
                eng.submit(sl[:T])
            eng.collect(want=False)
            eng.collect(want=False)
        eng.sync()
        barrier(dist, torch)
        t0 = time.perf_counter()
        inflight = 0
        for _ in range(args.steps):
            if inflight == 2:
                eng.collect(want=True)
                inflight -= 1
            eng.submit(eng.input_slot()[:T] if kind == "pinned" else src)
            inflight += 1
        while inflight:
            eng.collect(want=True)
            inflight -= 1
        eng.sync()
        barrier(dist, torch)
        sec = max_over_ranks(time.perf_counter() - t0, dist, torch)
        res[kind] = (aggregate_rate(B * Ch * T, 1 if dist is None else dist.get_world_size(), args.steps, sec),
                     1000.0 * sec / args.steps)
    return {"value": round(res["pinned"][0], 1), "unit": "frames/s", "ms_per_step": round(res["pinned"][1], 3),
            "pageable_value": round(res["pageable"][0], 1), "pageable_ms_per_step": round(res["pageable"][1], 3),
            "input_bytes_per_step": int(src.nbytes),
            "note": "streaming submit/collect, 2 pushes in flight: input from pinned host slots (value) or "
                    "pageable host memory (pageable_value), H2D over PCIe inside the timed region and "
                    "overlapped with the previous push; per-tick outputs copied back every push"}


def main():
    args = parse()
    if args.pmc_json is None:
        args.pmc_json = os.path.join(ROOT, "profiles", "pmc_traffic%s.json" % ("" if args.mode == "staged" else
                                                                             "_" + args.mode))
    maybe_spawn(args)
    if args.cpu_stub:
        return stub_main(args)
    rank, world, local, dist, torch = dist_setup(args.gpus)
    import fvad
    from fvad import cost

    B, Ch, T = args.streams_per_gpu, args.channels, args.ticks
    model = fvad.Model(seed=1)
    base, _ = stream_partition(rank, B)

    def measure(mode):
        """warmup, then exactly args.steps pushes between barriers; max over ranks"""
        eng = fvad.Engine(model, B, Ch, device=local, max_ticks=T, mode=mode)
        if mode != "fused" and not args.no_vadm:
            eng.attach_vadm()  # VADMachine.run per window on the device: the full per-frame VAD path
        eng.load_synthetic(T, base=base)
        for _ in range(args.warmup):
            eng.run_resident(T)
        eng.sync()
        eng.clear_times()
        barrier(dist, torch)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            eng.run_resident(T)
        eng.sync()
        barrier(dist, torch)
        elapsed = max_over_ranks(time.perf_counter() - t0, dist, torch)
        return eng, elapsed, eng.kernel_times()

    eng, elapsed, kt = measure(args.mode)
    value = aggregate_rate(B * Ch * T, world, args.steps, elapsed)
    ms_per_step = 1000.0 * elapsed / args.steps

    host = host_rate(eng, args, rank, dist, torch) if args.host_rate else None
    variants = None
    if args.variants and args.mode == "staged":
        del eng  # one engine's buffers at a time
        _, el16, kt16 = measure("fp16")
        variants = {"fp16": {
            "value": round(aggregate_rate(B * Ch * T, world, args.steps, el16), 1), "unit": "frames/s",
            "ms_per_step": round(1000.0 * el16 / args.steps, 3),
            "dtype": "f32+f16 (GRU gates: f16 MFMA, f32 accumulate)",
            "k_gru16_ms": round(kt16["kernels"].get("k_gru16", 0.0), 4),
            "parity": "tolerance (SURVEY.md 8(c): vad |d| <= 2e-2, segments identical; tests/test_gpu_fp16.py)",
            "note": "BASELINE configs[4]'s fp16-GRU variant on the same workload and clock (bench.py --mode fp16 "
                    "gives its full line)"}}

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return

    # roofline of the dominant kernel, per launch, from HIP events recorded
    # around each kernel on the stream it runs on (fvad_engine_kernel_times)
    frames_launch = B * Ch * T
    if args.mode == "fused":
        prep_share = cost.phases(Ch)["prep: s16 scale + HP biquad + rms"]
        per_k = {"k_prep": {"flops": prep_share, "bytes": cost.prep_kernel_bytes(B, Ch, T) / frames_launch},
                 "k_frame": {"flops": cost.flops_per_channel_frame(Ch) - prep_share,
                             "bytes": cost.frame_kernel_bytes(B, Ch, T) / frames_launch}}
    else:
        per_k = cost.staged_kernels(Ch)
    ridge = FP32_PEAK_TFLOPS * 1e12 / (HBM_PEAK_GBS * 1e9)
    kernels = {}
    for name, ms in kt["kernels"].items():
        c = per_k[name]
        sec = ms / 1000.0
        kernels[name] = {"ms": round(ms, 4), "tflops": round(c["flops"] * frames_launch / sec / 1e12, 3),
                         "gbs": round(c["bytes"] * frames_launch / sec / 1e9, 1),
                         "intensity": round(c["flops"] / c["bytes"], 2) if c["bytes"] else None}
    # k_vadm_hbm (side stream, after the push) and k_prep3 (prep stream, beside
    # the previous push) are overlapped with the main stream's kernels: timed
    # and listed, but not candidates for the pipeline's bottleneck
    side = ("k_vadm_hbm", "k_prep3")
    dom = max((n for n in kt["kernels"] if n not in side), key=lambda n: kt["kernels"][n])
    c = per_k[dom]
    dom_s = kt["kernels"][dom] / 1000.0
    alg_flops = c["flops"] * frames_launch
    alg_bytes = c["bytes"] * frames_launch
    compute_bound = c["flops"] / c["bytes"] >= ridge
    traffic = None
    pmc_src = None
    push_bytes = None
    if os.path.exists(args.pmc_json):
        try:
            with open(args.pmc_json) as f:
                pm = json.load(f)
            if (pm.get("streams"), pm.get("ticks"), pm.get("channels"), pm.get("mode")) == (B, T, Ch, args.mode):
                traffic = pm.get("bytes_per_launch", {}).get(dom)
                pmc_src = os.path.relpath(args.pmc_json, ROOT)
                # every kernel of a push (the side-stream ones included)
                push_bytes = sum(v for n, v in pm.get("bytes_per_launch", {}).items() if n in kt["kernels"])
        except Exception:
            traffic = None
    if compute_bound:
        achieved, peak, unit = alg_flops / dom_s / 1e12, FP32_PEAK_TFLOPS, "TFLOP/s"
    else:
        achieved, peak, unit = alg_bytes / dom_s / 1e9, HBM_PEAK_GBS, "GB/s"
    # whole path: frames/s against the lower of the HBM and
    # FP32-VALU ceilings for the path's algorithmic bytes / flops per frame
    f_alg = cost.flops_per_channel_frame(Ch)
    b_alg = cost.path_bytes_per_channel_frame(Ch)
    fps_gpu = value / world
    ceil_hbm = HBM_PEAK_GBS * 1e9 / b_alg
    ceil_valu = FP32_PEAK_TFLOPS * 1e12 / f_alg
    path = {"f_alg": round(f_alg), "b_alg": round(b_alg), "frames_per_s_per_gpu": round(fps_gpu, 1),
            "ceiling_hbm": round(ceil_hbm, 1), "ceiling_valu": round(ceil_valu, 1),
            "bound": "hbm" if ceil_hbm < ceil_valu else "valu",
            "frac": round(fps_gpu / min(ceil_hbm, ceil_valu), 5),
            "hbm_frac_alg": round(fps_gpu * b_alg / (HBM_PEAK_GBS * 1e9), 5),
            "valu_frac": round(fps_gpu * f_alg / (FP32_PEAK_TFLOPS * 1e12), 5)}
    roofline = {
        "bound": "valu" if compute_bound else "hbm",
        "roof": ("FP32 VALU (157.3 TFLOP/s; no MFMA instruction runs on this path)"
                 if compute_bound else "HBM3E 8 TB/s"),
        "kernel": dom,
        "achieved": round(achieved, 4), "peak": peak, "unit": unit, "frac": round(achieved / peak, 5),
        "traffic": traffic, "traffic_source": pmc_src,
        "alg_flops_per_launch": alg_flops, "alg_bytes_per_launch": alg_bytes,
        "flop_counts": "fvad/cost.py, data-dependent trip counts instrumented in the oracle (%s)" % (
            ", ".join("%s %s" % kv for kv in cost.MEASURED.items())),
        "kernel_ms_avg": round(kt["kernels"][dom], 4), "push_ms_avg": round(kt["total_ms"], 4),
        "timed_launches": kt["runs"],
        "path": path,
        "kernels": kernels,
    }
    if push_bytes:
        # whole-push HBM traffic (PMC bytes of all its kernels) over the
        # measured time per push: the pipeline's average HBM utilisation
        gbs = push_bytes / (ms_per_step / 1000.0) / 1e9
        roofline["push_hbm"] = {"bytes": push_bytes, "gbs": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4),
                                "bytes_per_frame": round(push_bytes / frames_launch, 1)}
    cpu = None
    if args.cpu_baseline and world == 1:
        try:
            cpu = cpu_baseline(args)
        except Exception as ex:  # never let the baseline leg kill the GPU measurement
            cpu = {"value": None, "unit": "frames/s", "cores": 0, "kind": "port", "sample": "failed: %s" % ex}
    line = {
        "metric": METRIC, "value": round(value, 1), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32" if args.mode != "fp16" else "f32+f16 (GRU gates: f16 MFMA, f32 accumulate)",
        "data": "synthetic",
        "config": {"workload": "configs[4] per-GPU partition: %d synthetic 48 kHz streams x %d ch per GPU "
                               "(%d at %d GPU), %d ticks (480 samples/ch) per step, %s"
                               % (B, Ch, B * world, world, T,
                                  "fp16 GRU weights on MFMA (configs[4] variant, tolerance parity)" if args.mode == "fp16"
                                  else "fp32 weights, bit-exact path"),
                   "streams_per_gpu": B, "channels": Ch, "ticks_per_step": T, "fft_size": 2048,
                   "parallelism": "stream-partition x%d (no collectives)" % world, "mode": args.mode,
                   "vad_machine": "device" if (args.mode != "fused" and not args.no_vadm) else "none"},
        "realtime_streams": round(value / (100.0 * Ch), 1),
        "roofline": roofline,
        "cpu_baseline": cpu,
    }
    if variants is not None:
        line["variants"] = variants
    if host is not None:
        line["host_buffers"] = host
        line["realtime_streams_host"] = round(host["value"] / (100.0 * Ch), 1)
    print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
