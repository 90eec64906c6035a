#!/usr/bin/env python3
"""Bench: Formula-VAD per-frame hot path on MI355X.

Metric (BASELINE.json): 48 kHz 480-sample VAD frames/sec whole node; max
concurrent real-time streams.  A VAD frame = one 480-sample channel-frame
through rnnoise (+ its share of the 2048-point band-energy FFT).

Workload: configs[4]'s per-GPU partition — 2048 synthetic 48 kHz stereo
streams per GPU (16384 at 8 GPUs), weak scaling, f32 exact numerics.  A step
= one push of TICKS ticks (480 samples per channel) for every stream of the
partition — the staged pipeline's kernels (fvad_staged.hip; --mode fused:
k_prep + k_frame) on the engine's HIP streams, device VADMachine included.
The input is RESIDENT_PUSHES distinct pushes (default 20 x 0.5 s = the first
10 s of every stream: burst onsets, speech, the every-20th-stream digital
silence at t = 5 s) held in HBM and cycled through push by push; with the
driver's --warmup 5 --steps 20 the timed pushes are exactly one cycle, the
input the flop counts of fvad/cost.py MEASURED were instrumented on.

Multi-GPU: one process per GPU.  Under torch.distributed.run (WORLD_SIZE set)
each rank runs its own stream partition; `--gpus N` without WORLD_SIZE
re-launches this script under torch.distributed.run with N ranks as a child
process, before anything touches the GPU.  The only collectives are the
barrier and the max-reduce of the timing (no data-path collective), on a
gloo process group with CPU tensors: no RCCL communicator or torch HIP stream
takes a hardware queue from the engine.

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
F16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: ~2.5 PF dense BF16/FP16 MFMA (no 2:1 sparsity)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # a timed region starts with no push in flight, so its first push runs its
    # k_prep3 (~2.5 ms) unoverlapped: ~2 % of 20 steps.  warmup 5 + steps 20
    # make the timed pushes exactly one cycle of the 20 resident pushes
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--resident-pushes", type=int, default=20,
                    help="distinct pushes of synthetic input resident in HBM, cycled through (20 = 10 s)")
    ap.add_argument("--streams-per-gpu", type=int, default=2048)
    ap.add_argument("--channels", type=int, default=2)
    ap.add_argument("--ticks", type=int, default=50)
    ap.add_argument("--mode", choices=("staged", "fused", "fp16", "fp16_fused"), default="staged",
                    help="staged (bit-exact, default), fused (bit-exact), fp16 (configs[4]: GRU on MFMA, tolerance), "
                         "fp16_fused (configs[4]'s fused FFT -> feature -> GRU kernel, k_fused16; equal to fp16)")
    ap.add_argument("--no-vadm", action="store_true", help="staged: do not run the device VADMachine (k_vadm)")
    ap.add_argument("--cpu-baseline", type=int, default=1, help="time the CPU oracle on this host (rank 0)")
    ap.add_argument("--cpu-streams", type=int, default=48,
                    help="CPU sample: streams 0..N-1 of this rank's partition (every 20th has digital silence)")
    ap.add_argument("--cpu-ticks", type=int, default=0,
                    help="CPU sample: ticks per stream (0: the whole resident cycle the GPU times)")
    ap.add_argument("--cpu-seconds", type=float, default=8.0,
                    help="measure each CPU sample (single-core, all-core) for about this long")
    ap.add_argument("--pmc-json", default=None,
                    help="PMC byte counts (tools/profile.sh); default profiles/pmc_traffic[_<mode>].json")
    ap.add_argument("--host-rate", type=int, default=1,
                    help="also time pushes from host buffers (PCIe-inclusive; reported as host_buffers, never value)")
    ap.add_argument("--cpu-stub", action="store_true",
                    help="no GPU: gloo ranks with a stub engine (tests the launcher, barrier and max-reduce)")
    ap.add_argument("--rehearse-on-gpu0", action="store_true",
                    help="multi-rank rehearsal on a 1-GPU box: every rank's engine on device 0, otherwise the "
                         "code the driver runs at N > 1 (gloo collectives on the CPU); the ranks share one GPU, so "
                         "the rate is no scaling figure and the line says so")
    ap.add_argument("--groups", type=int, default=1,
                    help="engines per GPU (fvad.EngineGroup): the rank's streams split into this many "
                         "sub-partitions pushing concurrently, k_prep3 / VADMachines on shared side streams "
                         "(opt-in: the gain depends on the runtime's hardware-queue placement, DESIGN.md 8 r5)")
    ap.add_argument("--one-engine-leg", type=int, default=1,
                    help="with --groups > 1, also time one engine over all the rank's streams "
                         "(roofline.one_engine: each kernel alone on the GPU)")
    ap.add_argument("--variants", type=int, default=1,
                    help="staged runs: also time the fp16 engine mode (configs[4]'s variant) on the same "
                         "workload and report it under `variants` (never `value`)")
    a = ap.parse_args()
    if a.groups < 1 or a.streams_per_gpu % a.groups:
        ap.error("--groups must divide --streams-per-gpu")
    return a


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


def dist_setup(n_gpus):
    """One process per GPU (torch.distributed.run env).  The process group is
    gloo at every N, its tensors on the CPU: the only collectives are the
    timing barrier, the max-reduce and the kernel-table gather, so no RCCL
    communicator and no torch HIP stream competes with the engine's streams
    for the GPU's hardware queues (GPU_MAX_HW_QUEUES = 4).
    Initialised whenever torch.distributed.run launched this process (world 1
    included).  Under torch.distributed.run the world size is the launcher's;
    it must match --gpus when that was given explicitly."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if n_gpus > 1 and world != n_gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d" % (n_gpus, world))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if "WORLD_SIZE" in os.environ:
        import torch
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo")
        return rank, world, local, dist, torch
    return rank, world, local, None, None


def barrier(dist, torch):
    if dist is not None:
        dist.barrier()


def max_over_ranks(x, dist, torch):
    if dist is None:
        return x
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def stream_partition(rank, streams_per_gpu):
    """Weak scaling: rank r owns synthetic stream ids [r*B, (r+1)*B) (configs[3]/[4]);
    streams are independent, so there is no data-path collective."""
    return rank * streams_per_gpu, streams_per_gpu


RSS_STAGES = {}
RSS_ANON = {}


def rss_stage(name):
    """This process's resident set (MB) at a named stage (host_memory.stages):
    VmRSS, and RssAnon (the heap: what the pinned slots, which the kernel
    driver maps and counts as file / shared pages, are not part of)."""
    try:
        with open("/proc/self/status") as f:
            kb = {ln.split(":")[0]: int(ln.split()[1]) for ln in f if ln.startswith(("VmRSS:", "RssAnon:"))}
        RSS_STAGES[name] = round(kb["VmRSS"] / 1024.0, 1)
        if "RssAnon" in kb:
            RSS_ANON[name] = round(kb["RssAnon"] / 1024.0, 1)
    except (OSError, KeyError, ValueError, IndexError):
        pass


def aggregate_rate(frames_per_rank_step, world, steps, elapsed_max):
    """Whole-job channel-frames/s: every rank's frames over the slowest rank's time."""
    return frames_per_rank_step * world * steps / elapsed_max


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            return next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), "")
    except OSError:
        return ""


def cpu_baseline(args, base=0):
    """The oracle's whole per-stream path (rnnoise + re-block + FFT B band sums
    + VADMachine: ora_bench_pipeline, the same work scope as the GPU step),
    built -O3 -march=native -ffp-contract=off on this host, one OS thread per
    group of streams (simulator.zig:217-228 runs one per instance).  Timed
    single-core and on every CPU this process may use, capped at 16: the GPU
    box allots 16 of its host's hardware threads to one GPU and asks worker
    pools to stay within that share.  Bounded sample: the whole resident cycle
    the GPU times (10 s: burst onsets, speech, the every-20th-stream digital
    silence at t = 5 s) of the partition's first CPU_STREAMS streams, pushed in
    50-tick chunks like the GPU step, repeated for about --cpu-seconds each.
    A whole-host figure (per-thread rate x the host's hardware threads) is
    reported as an extrapolation, never as `value`."""
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
    total = args.resident_pushes * args.ticks
    S, T, Ch = min(args.cpu_streams, args.streams_per_gpu), args.cpu_ticks or total, args.channels
    n = T * 480
    pcm = np.zeros((S, Ch, n), np.float32)
    for s in range(S):
        x, _ = fvad.synth_stream(base + s, total * 480, Ch)  # the resident input's generator length
        pcm[s] = x[:, :n]

    def timed(nthr, streams):
        secs, reps = 0.0, 0
        while secs < args.cpu_seconds and reps < 200:
            dt, _ = oracle.bench_pipeline(pcm[:streams], chunk=args.ticks * 480, n_threads=nthr, L=L)
            secs += dt
            reps += 1
        return streams * T * Ch * reps / secs, secs, reps

    one, one_s, one_r = timed(1, max(1, S // 16))
    allc, all_s, all_r = timed(threads, S)
    hw = os.cpu_count() or threads
    return {"value": round(allc, 1), "unit": "frames/s", "cores": threads, "kind": "port",
            "single_core": round(one, 1),
            "host_threads": hw,
            "whole_host_extrapolated": round(allc / threads * hw, 1),
            "sample": "oracle whole path (rnnoise, FFT B band sums, VADMachine), -O3 -march=native "
                      "-ffp-contract=off on %s; %d threads = this GPU's CPU allotment on a host of %d hardware "
                      "threads (%d usable by this process; whole_host_extrapolated = per-thread rate x %d, not "
                      "measured); sample: %d ticks (%.1f s%s) of streams %d..%d of the %d x %d ch, "
                      "%d passes in %.1f s; single-core: %d streams, %d passes, %.1f s" % (
                          cpu_model, threads, hw, avail, hw, T, T * 0.01,
                          ", the GPU's whole resident cycle" if T == total else "", base, base + S - 1,
                          args.streams_per_gpu, Ch, all_r, all_s, max(1, S // 16), one_r, one_s)}


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
    rank, world, local, dist, torch = dist_setup(args.gpus)
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
    # stand-in kernel table: rank r's k_a takes 1 + r ms, k_b 2 - r ms
    kt = {"total_ms": 3.0, "runs": args.steps, "kernels": {"k_a": 1.0 + rank, "k_b": 2.0 - rank}}
    kt, ranks = gather_kernel_tables(kt, dist, torch, rank)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": aggregate_rate(B * Ch * T, world, args.steps, elapsed),
                          "unit": "frames/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": 1000.0 * elapsed / args.steps, "data": "stub (no GPU)",
                          "config": {"streams_per_gpu": B, "first_stream": base},
                          "roofline": {"kernels": kt["kernels"], "ranks": ranks}}), flush=True)
    if dist is not None:
        dist.destroy_process_group()


DEPTH = 3  # FVAD_MAX_IN_FLIGHT (include/fvad.h)


def host_rate(grp, args, rank, dist, torch, base):
    """Streaming from host memory (fvad_engine_input_slot / submit / collect):
    FVAD_MAX_IN_FLIGHT = 3 pushes in flight per engine of the group, the
    input's H2D copy over PCIe overlapping the earlier pushes' kernels,
    outputs copied back every push.  Input: the first two pushes of the
    resident synthetic audio, alternating.  pinned: the producer writes each
    push into the engines' pinned slots (the copy cost of the producer itself
    is not counted); pageable: submit from ordinary host arrays (plus a
    threaded copy into the slot); pinned_i16: the same audio as 16-bit samples
    through fvad_engine_input_slot_i16 / submit_i16 (half the PCIe bytes,
    converted on the device)."""
    import fvad
    import numpy as np
    es = grp.engines
    Ch, T = args.channels, args.ticks
    # host memory stays bounded: the two pushes are generated straight into the
    # pinned slots, the 16-bit slots are converted from them a tick at a time,
    # and the pageable leg's host arrays (push 0's audio, submitted every step)
    # live only during that leg
    slots = [[] for _ in es]
    for k in range(DEPTH):  # slot k holds push k & 1
        for g, e in enumerate(es):
            sl = e.input_slot()[:T]
            if k < 2:
                fvad.synth_ticks(base + grp.first[g], grp.sizes[g], Ch, args.resident_pushes * T, k * T, T, out=sl)
            else:
                sl[...] = slots[g][0]
            slots[g].append(sl)
            e.submit(sl)
    for _ in range(DEPTH):
        for e in es:
            e.collect(want=False)
    grp.sync()
    res = {}
    for kind in ("pinned", "pageable", "pinned_i16"):
        pages = None
        if kind == "pageable":
            pages = [np.array(sg[0]) for sg in slots]
        elif kind == "pinned_i16":
            for k in range(DEPTH):  # the same audio as 16-bit samples, slot by slot
                for g, e in enumerate(es):
                    sl16 = e.input_slot_i16()[:T]
                    for t in range(T):
                        sl16[t] = np.clip(np.round(slots[g][k][t] * np.float32(32768.0)), -32768, 32767)
                    e.submit_i16(sl16)
            for _ in range(DEPTH):
                for e in es:
                    e.collect(want=False)
        grp.sync()
        barrier(dist, torch)
        t0 = time.perf_counter()
        inflight = 0
        for k in range(args.steps):
            if inflight == DEPTH:
                for e in es:
                    e.collect(want=True)
                inflight -= 1
            for g, e in enumerate(es):
                if kind == "pinned_i16":
                    e.submit_i16(e.input_slot_i16()[:T])
                else:
                    e.submit(e.input_slot()[:T] if kind == "pinned" else pages[g])
            inflight += 1
        while inflight:
            for e in es:
                e.collect(want=True)
            inflight -= 1
        grp.sync()
        barrier(dist, torch)
        sec = max_over_ranks(time.perf_counter() - t0, dist, torch)
        # the same stream in steady state: W + K pushes back to back, timed from
        # the completion (collect) of push W - 1 to that of push W + K - 1 --
        # K push periods with the pipeline full, no fill or drain (a continuous
        # ingest's rate; the line above starts and ends with nothing in flight)
        W = DEPTH + 2
        done = []
        inflight = 0
        for k in range(W + args.steps):
            if inflight == DEPTH:
                for e in es:
                    e.collect(want=True)
                done.append(time.perf_counter())
                inflight -= 1
            for g, e in enumerate(es):
                if kind == "pinned_i16":
                    e.submit_i16(e.input_slot_i16()[:T])
                else:
                    e.submit(e.input_slot()[:T] if kind == "pinned" else pages[g])
            inflight += 1
        while inflight:
            for e in es:
                e.collect(want=True)
            done.append(time.perf_counter())
            inflight -= 1
        grp.sync()
        barrier(dist, torch)
        steady = max_over_ranks(done[W + args.steps - 1] - done[W - 1], dist, torch)
        rss_stage("host_" + kind)
        res[kind] = (aggregate_rate(grp.B * Ch * T, 1 if dist is None else dist.get_world_size(), args.steps, sec),
                     1000.0 * sec / args.steps, 1000.0 * steady / args.steps)
    in_bytes = sum(int(sg[0].nbytes) for sg in slots)
    return {"value": round(res["pinned"][0], 1), "unit": "frames/s", "ms_per_step": round(res["pinned"][1], 3),
            "pageable_value": round(res["pageable"][0], 1), "pageable_ms_per_step": round(res["pageable"][1], 3),
            "i16_value": round(res["pinned_i16"][0], 1), "i16_ms_per_step": round(res["pinned_i16"][1], 3),
            "steady_ms_per_step": {k: round(v[2], 3) for k, v in res.items()},
            "input_bytes_per_step": in_bytes, "i16_input_bytes_per_step": in_bytes // 2,
            "note": "streaming submit/collect, 3 pushes in flight per engine, input = the first two pushes of the "
                    "synthetic streams alternating: from pinned host slots (value) or pageable host arrays holding "
                    "the first push (pageable_value), H2D over PCIe inside the timed region and overlapped with "
                    "the previous push; per-tick outputs copied back every push; i16_value: the same audio as "
                    "16-bit samples from the pinned 16-bit slots (fvad_engine_submit_i16, k / 32768 converted on "
                    "the device).  steady_ms_per_step: the same streams with the pipeline kept full -- push "
                    "periods from one collect to the one %d pushes later, after %d pushes of warm-up (the "
                    "*_ms_per_step figures start and end with nothing in flight, so they include the first "
                    "push's H2D copy and k_prep3 and the last push's drain)" % (args.steps, DEPTH + 2)}


def gather_kernel_tables(kt, dist, torch, rank):
    """Every rank's per-kernel event times; the line reports the max over ranks
    per kernel (the slowest rank sets the step) and which rank that was."""
    if dist is None:
        return kt, None
    tables = [None] * dist.get_world_size()
    dist.all_gather_object(tables, {"rank": rank, "kt": kt})
    worst = {"total_ms": max(t["kt"]["total_ms"] for t in tables), "runs": min(t["kt"]["runs"] for t in tables),
             "kernels": {}}
    where = {}
    for name in kt["kernels"]:
        r = max(tables, key=lambda t: t["kt"]["kernels"].get(name, 0.0))
        worst["kernels"][name] = r["kt"]["kernels"].get(name, 0.0)
        where[name] = r["rank"]
    per_rank = {str(t["rank"]): {"push_ms_avg": round(t["kt"]["total_ms"], 4),
                                 "kernels": {k: round(v, 4) for k, v in t["kt"]["kernels"].items()}} for t in tables}
    return worst, {"max_rank": where, "per_rank": per_rank}


def main():
    args = parse()
    if args.pmc_json is None:
        args.pmc_json = os.path.join(ROOT, "profiles", "pmc_traffic%s.json" % ("" if args.mode == "staged" else
                                                                             "_" + args.mode))
    maybe_spawn(args)
    if args.cpu_stub:
        return stub_main(args)
    rank, world, local, dist, torch = dist_setup(args.gpus)
    if args.rehearse_on_gpu0:
        local = 0
    import fvad
    from fvad import cost

    B, Ch, T, P = args.streams_per_gpu, args.channels, args.ticks, args.resident_pushes
    model = fvad.Model(seed=1)
    base, _ = stream_partition(rank, B)

    def measure(mode, lt_full=False, groups=None):
        """warmup, then exactly args.steps pushes between barriers; max over ranks.
        The rank's streams as `groups` engines pushing concurrently
        (fvad.EngineGroup).  lt_full: the device VADMachines start as in a
        stream past its first long_term_speech_avg_sec (every long-term entry
        pushed; timing hook FVAD_DEBUG_VADM_LT_FULL, values not the reference's)"""
        groups = args.groups if groups is None else groups
        leg = mode + ("_lt_full" if lt_full else "") + ("_g%d" % groups if groups != args.groups else "")
        vadm = mode != "fused" and not args.no_vadm  # VADMachine.run per window on the device
        e = fvad.EngineGroup(model, B, Ch, groups=groups, vadm=vadm, device=local, max_ticks=T, mode=mode)
        rss_stage("engine_%s" % leg)
        if vadm and lt_full:
            e.set_debug(fvad.DEBUG_VADM_LT_FULL, 1)
        e.load_synthetic(T, base=base, pushes=P)
        rss_stage("resident_input_%s" % leg)
        for _ in range(args.warmup):
            e.run_resident(T)
        e.sync()
        e.clear_times()
        barrier(dist, torch)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            e.run_resident(T)
        e.sync()
        barrier(dist, torch)
        elapsed = max_over_ranks(time.perf_counter() - t0, dist, torch)
        return e, elapsed, e.kernel_times()

    rss_stage("start")
    eng, elapsed, kt_local = measure(args.mode)
    rss_stage("after_timed_%s" % args.mode)
    kt, ranks = gather_kernel_tables(kt_local, dist, torch, rank)
    value = aggregate_rate(B * Ch * T, world, args.steps, elapsed)
    ms_per_step = 1000.0 * elapsed / args.steps

    host = host_rate(eng, args, rank, dist, torch, base) if args.host_rate else None
    rss_stage("after_host_buffers")
    del eng  # one engine group's buffers at a time
    one = None
    if args.groups > 1 and args.one_engine_leg:
        # the same workload on one engine per GPU: its kernels run alone, so
        # their events give the isolated per-launch roofline beside the
        # co-running one of the line's own run
        e1, el1, kt1 = measure(args.mode, groups=1)
        del e1
        kt1, _ = gather_kernel_tables(kt1, dist, torch, rank)
        one = (el1, kt1)
    variants = None
    if args.variants and args.mode == "staged":
        e16, el16, kt16 = measure("fp16")
        del e16
        kt16, _ = gather_kernel_tables(kt16, dist, torch, rank)
        variants = {"fp16": {
            "value": round(aggregate_rate(B * Ch * T, world, args.steps, el16), 1), "unit": "frames/s",
            "ms_per_step": round(1000.0 * el16 / args.steps, 3),
            "dtype": "f32+f16 (GRU gates: f16 MFMA, f32 accumulate)",
            "k_gru16_ms": round(kt16["kernels"].get("k_gru16", 0.0), 4),
            "kernels_ms": {k: round(v, 4) for k, v in kt16["kernels"].items()},
            "parity": "tolerance (SURVEY.md 8(c): vad |d| <= 2e-2, segments identical or reported -- on this "
                      "workload under this schedule max |dvad| 8.5e-5 and one segment bound of 2048 streams "
                      "moved by one FFT-B window; tests/test_gpu_fullsize.py, test_gpu_fp16.py)",
            "note": "BASELINE configs[4]'s fp16-GRU variant on the same workload and clock (bench.py --mode fp16 "
                    "gives its full line)"}}
        ef, elf, ktf = measure("fp16_fused")
        del ef
        ktf, _ = gather_kernel_tables(ktf, dist, torch, rank)
        variants["fp16_fused"] = {
            "value": round(aggregate_rate(B * Ch * T, world, args.steps, elf), 1), "unit": "frames/s",
            "ms_per_step": round(1000.0 * elf / args.steps, 3),
            "dtype": "f32+f16 (GRU gates: f16 MFMA, f32 accumulate)",
            "k_fused16_ms": round(ktf["kernels"].get("k_fused16", 0.0), 4),
            "kernels_ms": {k: round(v, 4) for k, v in ktf["kernels"].items() if k != "k_pspecw"},
            "parity": "every output identical to the fp16 variant's (tests/test_gpu_fused16.py), so the fp16 "
                      "variant's tolerance parity holds",
            "note": "BASELINE configs[4]'s fused FFT -> feature -> GRU kernel: the pitch-spectrum FFT, its "
                    "features and the GRU stack in one kernel (k_fused16 in place of k_pspecw + k_gru16), same "
                    "workload and clock (bench.py --mode fp16_fused gives its full line)"}
        if not args.no_vadm:
            # the same workload with the VADMachines in their long-running
            # regime: a stream past its first 180 s re-folds a long-term
            # buffer of pushed values; timing only
            elt, ellt, ktlt = measure("staged", lt_full=True)
            del elt
            ktlt, _ = gather_kernel_tables(ktlt, dist, torch, rank)
            variants["long_running_streams"] = {
                "value": round(aggregate_rate(B * Ch * T, world, args.steps, ellt), 1), "unit": "frames/s",
                "ms_per_step": round(1000.0 * ellt / args.steps, 3),
                "kernels_ms": {k: round(v, 4) for k, v in ktlt["kernels"].items()},
                "note": "staged mode, the same input and clock, the device VADMachines started as in streams past "
                        "their first long_term_speech_avg_sec (180 s: every long-term entry a pushed value, timing "
                        "hook FVAD_DEBUG_VADM_LT_FULL; the VADMachine's values then are not the reference's).  "
                        "`value` covers streams in their first seconds, where the long-term buffer still holds "
                        "initial entries"}
    # host memory of this rank after its GPU legs (bounded: the synthetic input
    # is generated and uploaded 64 streams at a time, nothing cached; the
    # pinned slots of the streaming leg are FVAD_MAX_IN_FLIGHT pushes each way)
    import resource
    host_mem = {"peak_rss_mb": round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024.0, 1),
                "pinned_slots_mb": round(DEPTH * (B * Ch * T * 480 * 6 + B * T * 4 * 8) / 2 ** 20, 1)
                if args.host_rate else 0.0, "stages_rss_mb": dict(RSS_STAGES),
                "stages_anon_mb": dict(RSS_ANON)}
    host_mem_all = None
    if dist is not None:
        host_mem_all = [None] * world
        dist.all_gather_object(host_mem_all, host_mem)

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return

    line = {
        "metric": METRIC, "value": round(value, 1), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32" if args.mode not in ("fp16", "fp16_fused") else "f32+f16 (GRU gates: f16 MFMA, f32 accumulate)",
        "data": "synthetic" + ("; REHEARSAL: %d ranks sharing GPU 0 over gloo (--rehearse-on-gpu0), not a "
                               "scaling figure" % world if args.rehearse_on_gpu0 else ""),
        "config": {"workload": "configs[4] per-GPU partition: %d synthetic 48 kHz streams x %d ch per GPU "
                               "(%d at %d GPU), %d ticks (480 samples/ch) per step, %d distinct resident pushes "
                               "(%.1f s of every stream) cycled, %s"
                               % (B, Ch, B * world, world, T, P, P * T * 0.01,
                                  "fp16 GRU weights on MFMA (configs[4] variant, tolerance parity)" if args.mode in ("fp16", "fp16_fused")
                                  else "fp32 weights, bit-exact path"),
                   "streams_per_gpu": B, "channels": Ch, "ticks_per_step": T, "resident_pushes": P,
                   "fft_size": 2048,
                   "parallelism": "stream-partition x%d (no collectives), %d engines per GPU" % (world, args.groups),
                   "engines_per_gpu": args.groups, "mode": args.mode,
                   "vad_machine": "device" if (args.mode != "fused" and not args.no_vadm) else "none",
                   },
        "realtime_streams": round(value / (100.0 * Ch), 1),
        "roofline": roofline(args, kt, value, world, ms_per_step, cost, ranks),
        "engines_per_gpu": args.groups,
        "cpu_baseline": None,
    }
    if one is not None:
        el1, kt1 = one
        v1 = aggregate_rate(B * Ch * T, world, args.steps, el1)
        r1 = roofline(args, kt1, v1, world, 1000.0 * el1 / args.steps, cost, None, groups=1)
        line["roofline"]["one_engine"] = {
            "value": round(v1, 1), "ms_per_step": round(1000.0 * el1 / args.steps, 3),
            "kernel": r1.get("kernel"), "achieved": r1.get("achieved"), "frac": r1.get("frac"),
            "frac_attainable": r1.get("frac_attainable"), "kernel_ms_avg": r1.get("kernel_ms_avg"),
            "traffic": r1.get("traffic"), "kernels_ms": {k: v["ms"] for k, v in r1.get("kernels", {}).items()},
            "note": "the same workload on ONE engine per GPU (%d streams per launch), measured in its own leg: "
                    "each kernel alone on the GPU.  The line's value runs %d engines of %d streams whose kernels "
                    "co-run, so its per-launch times (roofline.kernels) include sharing the GPU with the other "
                    "engines' kernels" % (B, args.groups, B // args.groups)}
    line["host_memory"] = dict(host_mem, **({"per_rank_peak_rss_mb": [h["peak_rss_mb"] for h in host_mem_all]}
                                            if host_mem_all else {}))
    if variants is not None:
        line["variants"] = variants
    if host is not None:
        line["host_buffers"] = host
        line["realtime_streams_host"] = round(host["value"] / (100.0 * Ch), 1)
        line["realtime_streams_host_i16"] = round(host["i16_value"] / (100.0 * Ch), 1)
    if args.cpu_baseline:  # rank 0 only, at any N (the other ranks have finished)
        try:
            line["cpu_baseline"] = cpu_baseline(args, base)
        except Exception as ex:  # never let the baseline leg kill the GPU measurement
            line["cpu_baseline"] = {"value": None, "unit": "frames/s", "cores": 0, "kind": "port",
                                    "sample": "failed: %s" % ex}
    print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def roofline(args, kt, value, world, ms_per_step, cost, ranks, groups=None):
    """Roofline of the dominant kernel, per launch, from HIP events recorded
    around each kernel on the stream it runs on (fvad_engine_kernel_times; at
    N > 1 the max over ranks), plus the whole path against SURVEY.md 8(d)'s
    ceilings.  The engine records the events on every 4th timed push
    (FVAD_EVENT_EVERY): on every push their markers cost it ~1 %.  With
    `groups` engines per GPU a launch covers one engine's streams (B / groups)
    and co-runs with the other engines' kernels."""
    groups = args.groups if groups is None else groups
    Ball, Ch, T = args.streams_per_gpu, args.channels, args.ticks
    B = Ball // groups  # streams per launch (the bench's B is a multiple of groups)
    frames_launch = B * Ch * T
    if args.mode == "fused":
        prep_share = cost.phases(Ch)["prep: s16 scale + HP biquad + rms"]
        per_k = {"k_prep": {"flops": prep_share, "bytes": cost.prep_kernel_bytes(B, Ch, T) / frames_launch},
                 "k_frame": {"flops": cost.flops_per_channel_frame(Ch) - prep_share,
                             "bytes": cost.frame_kernel_bytes(B, Ch, T) / frames_launch}}
    else:
        per_k = cost.staged_kernels(Ch)
    if not any(ms > 0 for ms in kt["kernels"].values()):
        # FVAD_NO_EVENTS=1 (diagnostic): no per-kernel events were recorded
        return {"bound": None, "note": "no kernel timing events (FVAD_NO_EVENTS=1)", "kernels": {}}
    # bit-exact C-order sums: no product may fuse with its sum (-ffp-contract=off),
    # so a flop is one lane-op and the attainable FP32 VALU rate is half the
    # FMA-counted 157.3 TFLOP/s; a kernel is VALU-bound when its intensity
    # clears THAT ridge (9.8 flop/B), HBM-bound otherwise
    valu_nofma = FP32_PEAK_TFLOPS / 2
    ridge = valu_nofma * 1e12 / (HBM_PEAK_GBS * 1e9)
    kernels = {}
    for name, ms in kt["kernels"].items():
        c = per_k[name]
        if ms <= 0:  # not run (or not timed) in the timed pushes
            kernels[name] = {"ms": 0.0, "tflops": None, "gbs": None, "intensity": None}
            continue
        sec = ms / 1000.0
        kernels[name] = {"ms": round(ms, 4), "tflops": round(c["flops"] * frames_launch / sec / 1e12, 3),
                         "gbs": round(c["bytes"] * frames_launch / sec / 1e9, 1),
                         "intensity": round(c["flops"] / c["bytes"], 2) if c["bytes"] else None}
    # k_vadm_hbm (side stream, beside the next push), k_vadm_par (the last
    # push's machine, at the final sync) and k_prep3 (prep stream, beside the
    # previous push) run off the main stream: timed and listed, but not
    # candidates for the pipeline's bottleneck
    side = ("k_vadm_hbm", "k_vadm_par", "k_prep3")
    dom = max((n for n in kt["kernels"] if n not in side), key=lambda n: kt["kernels"][n])
    c = per_k[dom]
    dom_s = kt["kernels"][dom] / 1000.0
    alg_flops = c["flops"] * frames_launch
    alg_bytes = c["bytes"] * frames_launch
    intensity = c["flops"] / c["bytes"]
    compute_bound = intensity >= ridge
    traffic = None
    pmc_src = None
    push_bytes = None
    if os.path.exists(args.pmc_json):
        try:
            with open(args.pmc_json) as f:
                pm = json.load(f)
            if (pm.get("streams"), pm.get("ticks"), pm.get("channels"), pm.get("mode"),
                    pm.get("groups", 1)) == (Ball, T, Ch, args.mode, groups):
                traffic = pm.get("bytes_per_launch", {}).get(dom)
                pmc_src = os.path.relpath(args.pmc_json, ROOT)
                # every kernel of a push (the side-stream ones included), every engine
                push_bytes = groups * sum(v for n, v in pm.get("bytes_per_launch", {}).items()
                                          if n in kt["kernels"])
        except Exception:
            traffic = None
    if compute_bound:
        achieved, peak, unit = alg_flops / dom_s / 1e12, FP32_PEAK_TFLOPS, "TFLOP/s"
        attainable = min(valu_nofma, intensity * HBM_PEAK_GBS / 1000.0)
    else:
        achieved, peak, unit = alg_bytes / dom_s / 1e9, HBM_PEAK_GBS, "GB/s"
        attainable = HBM_PEAK_GBS
    # whole path: frames/s against the lower of the HBM and
    # FP32-VALU ceilings for the path's algorithmic bytes / flops per frame.
    # fp16 mode: the GRU stack's flops run on f16 MFMA (2.5 PFLOP/s dense,
    # v_mfma_f32_16x16x32_f16), the rest on the VALU
    f_alg = cost.flops_per_channel_frame(Ch)
    b_alg = cost.path_bytes_per_channel_frame(Ch)
    f_gru = cost.phases(Ch)["GRU stack"] if args.mode in ("fp16", "fp16_fused") else 0.0
    fps_gpu = value / world
    ceil_hbm = HBM_PEAK_GBS * 1e9 / b_alg
    ceil_valu = 1.0 / ((f_alg - f_gru) / (FP32_PEAK_TFLOPS * 1e12) + f_gru / (F16_MFMA_PEAK_TFLOPS * 1e12))
    path = {"f_alg": round(f_alg), "b_alg": round(b_alg), "frames_per_s_per_gpu": round(fps_gpu, 1),
            "ceiling_hbm": round(ceil_hbm, 1), "ceiling_valu": round(ceil_valu, 1),
            "bound": "hbm" if ceil_hbm < ceil_valu else "valu",
            "frac": round(fps_gpu / min(ceil_hbm, ceil_valu), 5),
            "hbm_frac_alg": round(fps_gpu * b_alg / (HBM_PEAK_GBS * 1e9), 5),
            "valu_frac": round(fps_gpu * f_alg / (FP32_PEAK_TFLOPS * 1e12), 5)}
    if f_gru:
        path["ceiling_note"] = ("fp16 mode: the GRU stack's %d flop per frame priced at the f16 MFMA peak "
                                "(%.0f TFLOP/s), the other %d at the FP32 VALU peak" % (
                                    f_gru, F16_MFMA_PEAK_TFLOPS, f_alg - f_gru))
    if compute_bound:
        roof = ("FP32 VALU (157.3 TFLOP/s, FMA-counted; %s)" %
                ("the GRU stack is on f16 MFMA, this kernel is not" if args.mode in ("fp16", "fp16_fused") and dom not in ("k_gru16", "k_fused16")
                 else "no MFMA instruction runs in this kernel"))
    else:
        roof = "HBM3E 8 TB/s"
    out = {
        "bound": "valu" if compute_bound else "hbm",
        "roof": roof,
        "kernel": dom,
        "achieved": round(achieved, 4), "peak": peak, "unit": unit, "frac": round(achieved / peak, 5),
        "attainable": round(attainable, 2), "frac_attainable": round(achieved / attainable, 5),
        "attainable_note": "min(FP32 VALU without FMA = 78.65 TFLOP/s, intensity x 8 TB/s) for a VALU-bound "
                           "kernel: the bit-exact C-order sums keep every mul and add separate",
        "traffic": traffic, "traffic_source": pmc_src,
        "alg_flops_per_launch": alg_flops, "alg_bytes_per_launch": alg_bytes,
        "flop_counts": "fvad/cost.py, data-dependent trip counts instrumented in the oracle (%s)" % (
            ", ".join("%s %s" % kv for kv in cost.MEASURED.items())),
        "kernel_ms_avg": round(kt["kernels"][dom], 4), "push_ms_avg": round(kt["total_ms"], 4),
        "timed_launches": kt["runs"],
        "event_sampling": "events on every %s-th timed push" % os.environ.get("FVAD_EVENT_EVERY", "4"),
        "path": path,
        "kernels": kernels,
    }
    if ranks is not None:
        out["ranks"] = ranks
        out["kernels_note"] = "max over ranks per kernel (ranks.max_rank names the rank)"
    if push_bytes:
        # whole-push HBM traffic (PMC bytes of all its kernels) over the
        # measured time per push: the pipeline's average HBM utilisation
        gbs = push_bytes / (ms_per_step / 1000.0) / 1e9
        out["push_hbm"] = {"bytes": push_bytes, "gbs": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4),
                           "bytes_per_frame": round(push_bytes / (groups * frames_launch), 1)}
    out["engines_per_gpu"] = groups
    out["streams_per_launch"] = B
    return out


if __name__ == "__main__":
    main()
