"""Parity at the sizes the bench times and the multi-GPU configs shard, every
stream against the CPU oracle (VAD.zig:214-348 frame loop, denoiser,
re-block, FFT B; VADMachine.zig:126-230 segments):

* the bench's exact timed workload (bench.py): 2048 stereo streams, 50-tick
  pushes, the 20 distinct resident pushes (the first 10 s of every stream:
  burst onsets, speech, the every-20th-stream digital silence at t = 5 s),
  device VADMachine attached; then five pushes streamed from host memory
  (submit / collect, three in flight) that replay the cycle's first 2.5 s, as
  the bench's second cycle does -- staged mode bit for bit, fp16 mode
  (configs[4]'s variant) at the stated tolerance;
* the bench's exact SCHEDULE (bench.py:387-401): the same 25 pushes through
  run_resident with no synchronisation between them -- the next push's
  k_prep3 overlapping this one's kernels, the steady-state k_vadm_hbm beside
  the next push, k_vadm_par only for the push before a sync -- every push's
  outputs (recorded on the device by fvad_engine_output_log, no host sync),
  every stream's segments, the whole VADMachine state (fvad_engine_vadm_snapshot)
  and its RollingAverage buffers against the oracle fed the same 25 pushes;
  also with every machine on k_vadm_par and a third of them forced through its
  in-kernel serial fallback, and with the lazy long-term bound made infinite
  (every test the estimate would settle folds exactly); the fp16 variant under
  the same schedule at its tolerance;
* configs[3]'s per-GPU shard: 4096 streams over 8 GPUs = 512 streams, here
  rank 3's ids 1536..2047, 12 pushes (6 s, the silence included), staged and
  fp16.

The oracle side of each workload is computed once per module (16 threads)
and shared by the staged and fp16 tests.
"""
import concurrent.futures as cf
import functools
import hashlib

import numpy as np
import pytest

import parity_util as pu

pytestmark = pytest.mark.gpu

FRAME = 480
T = 50
# test_gpu_fp16.py's bounds (vad |d| <= 2e-2)
VAD_ABS = 1e-3
BAND_REL = 2e-3
SEG_SHIFT = 4 * 2048  # fp16: a segment bound may move by at most 4 FFT-B windows


def _digest(a):
    return hashlib.sha1(np.ascontiguousarray(a, np.float64).tobytes()).hexdigest()


def _oracle_stream(args):
    import fvad
    import oracle
    sid, total_ticks, replay_ticks = args
    x = fvad.synth_stream(sid, total_ticks * FRAME, 2)[0]
    om = _om()
    frames = total_ticks + replay_ticks
    p = oracle.Pipeline(2, om, trace_frames=frames + 1, trace_windows=frames // 4 + 2)
    n = T * FRAME
    for a in range(0, total_ticks * FRAME, n):
        p.push([x[0, a:a + n], x[1, a:a + n]])
    for a in range(0, replay_ticks * FRAME, n):
        p.push([x[0, a:a + n], x[1, a:a + n]])
    fr, wi = p.trace()
    # the machine's whole state after every push, its long-term buffer (4218
    # entries) as a digest, the short ones as arrays
    state = (p.vadm_snapshot(), _digest(p.vadm_rolling(0)), p.vadm_rolling(1), p.vadm_rolling(2))
    return fr, wi, p.segments(), state


@functools.lru_cache(maxsize=None)
def _om():
    import oracle
    return oracle.Model(seed=1)


@functools.lru_cache(maxsize=None)
def oracle_workload(base, n_streams, pushes, replay_pushes):
    import oracle
    oracle.tables()
    _om()
    with cf.ThreadPoolExecutor(max_workers=16) as ex:
        return list(ex.map(_oracle_stream, [(base + s, pushes * T, replay_pushes * T) for s in range(n_streams)]))


def run_engine(fvad_mod, model, mode, base, n_streams, pushes, replay_pushes, want_state=False):
    """The bench's engine: resident cycle (run_resident), then the cycle's
    first replay_pushes pushes again through submit / collect."""
    eng = fvad_mod.Engine(model, n_streams, 2, max_ticks=T, mode=mode)
    eng.attach_vadm()
    eng.load_synthetic(T, base=base, pushes=pushes)
    outs = []
    for _ in range(pushes):
        eng.run_resident(T)
        eng.sync()
        outs.append(eng.fetch(T))
    if replay_pushes:
        # streamed, at most FVAD_MAX_IN_FLIGHT (3) uncollected
        src = fvad_mod.synth_ticks(base, n_streams, 2, pushes * T, 0, replay_pushes * T)
        inflight = 0
        for k in range(replay_pushes):
            if inflight == 3:
                outs.append(eng.collect())
                inflight -= 1
            eng.submit(src[k * T:(k + 1) * T])
            inflight += 1
        for _ in range(inflight):
            outs.append(eng.collect())
    eng.sync()
    got = {k: np.concatenate([o[k] for o in outs]) for k in outs[0]}
    segs = [eng.segments(s) for s in range(n_streams)]
    if want_state:
        return got, segs, device_state(eng, n_streams)
    return got, segs


def device_state(eng, n_streams):
    """Every stream's machine state and RollingAverage buffers (the oracle's form)."""
    return [(eng.vadm_snapshot(s), _digest(eng.vadm_rolling(s, 0)), eng.vadm_rolling(s, 1), eng.vadm_rolling(s, 2))
            for s in range(n_streams)]


def check_state(ref, got_state):
    for s, (r, g) in enumerate(zip(ref, got_state)):
        rs, gs = r[3], g
        assert rs[0] == gs[0], (s, rs[0], gs[0])
        assert rs[1] == gs[1], (s, "long-term RollingAverage buffer differs")
        assert np.array_equal(rs[2], gs[2]) and np.array_equal(rs[3], gs[3]), (s, "short RollingAverage buffers")


def check_exact(ref, got, segs):
    n_seg = 0
    for s, (fr, wi, rsegs, _) in enumerate(ref):
        assert np.array_equal(fr["vad"], got["vad"][:, s]), (s, pu.first_mismatch(fr["vad"], got["vad"][:, s]))
        assert np.array_equal(fr["ratio"], got["ratio"][:, s]), s
        wf = got["win_flag"][:, s].astype(bool)
        assert len(wi) == wf.sum(), s
        assert np.array_equal(wi["band"][:, :2], got["band"][wf, s, :, 0]), s
        assert np.array_equal(wi["ratio"], got["win_ratio"][wf, s]), s
        assert np.array_equal(wi["vad"], got["win_vad"][wf, s]), s
        assert segs[s] == rsegs, s
        n_seg += len(rsegs)
    return n_seg


MAX_MOVED = 3


def check_tolerance(ref, got, segs):
    worst_v, worst_b, n_seg, diffs = 0.0, 0.0, 0, []
    for s, (fr, wi, rsegs, _) in enumerate(ref):
        dv = float(np.abs(fr["vad"] - got["vad"][:, s]).max())
        assert dv <= VAD_ABS, (s, dv)
        assert np.array_equal(fr["ratio"], got["ratio"][:, s]), s  # computed before the GRU
        wf = got["win_flag"][:, s].astype(bool)
        assert len(wi) == wf.sum(), s
        assert np.array_equal(wi["ratio"], got["win_ratio"][wf, s]), s
        assert float(np.abs(wi["vad"] - got["win_vad"][wf, s]).max()) <= VAD_ABS, s
        b_ref, b_got = wi["band"][:, :2], got["band"][wf, s, :, 0]
        db = float(np.abs(b_ref - b_got).max() / max(1e-12, np.abs(b_ref).max()))
        assert db <= BAND_REL, (s, db)
        # segment bounds: identical, or reported (SURVEY.md 8(c) for this
        # config): a band sum within BAND_REL can still cross a VADMachine
        # threshold one window earlier or later
        a, b = [g[:2] for g in segs[s]], [g[:2] for g in rsegs]
        if a != b:
            assert len(a) == len(b), (s, a, b)
            shift = max(abs(int(x) - int(y)) for p, q in zip(a, b) for x, y in zip(p, q))
            assert shift <= SEG_SHIFT, (s, a, b)
            diffs.append((s, shift))
        worst_v, worst_b = max(worst_v, dv), max(worst_b, db)
        n_seg += len(rsegs)
    # the observed count plus a margin: 1 of the bench workload's 2048 streams
    # (one segment end one FFT-B window early), none of the 512-stream shard's
    assert len(diffs) <= MAX_MOVED, diffs
    return worst_v, worst_b, n_seg, diffs


@pytest.fixture(scope="module")
def model(fvad_mod):
    return fvad_mod.Model(seed=1)


BENCH = (0, 2048, 20, 5)      # base, streams, resident pushes, replayed pushes (25 = bench warmup 5 + steps 20)
SHARD = (1536, 512, 12, 0)    # configs[3]: rank 3 of 8, 512 streams, 6 s


@pytest.mark.timeout(900)
def test_bench_workload_staged_every_stream(fvad_mod, oracle_mod, model):
    """bench.py's timed input (the 20-push resident cycle) + two streamed
    replay pushes: every stream's vad, ratio, window flag / ratio / vad, band
    sums and segments equal the oracle's bit for bit."""
    got, segs, state = run_engine(fvad_mod, model, "staged", *BENCH, want_state=True)
    assert (got["vad"][500:600, 19::20] == 0).sum() > 5000  # the silent streams hit the E < 0.04 gate
    ref = oracle_workload(*BENCH)
    n_seg = check_exact(ref, got, segs)
    assert n_seg > 100
    check_state(ref, state)
    print("bench workload staged: 2048 streams x %d frames bit-exact, %d segments" % (len(ref[0][0]), n_seg))


@pytest.mark.timeout(900)
def test_bench_workload_fp16_every_stream(fvad_mod, oracle_mod, model):
    """The same workload in fp16 mode (configs[4]'s variant): every stream's
    vad within VAD_ABS, volume / window ratios bit-identical, band sums within
    BAND_REL; segment bounds identical except on at most 1 % of the streams,
    where a bound may move by at most SEG_SHIFT samples (reported)."""
    got, segs = run_engine(fvad_mod, model, "fp16", *BENCH)
    ref = oracle_workload(*BENCH)
    wv, wb, n_seg, diffs = check_tolerance(ref, got, segs)
    print("bench workload fp16: max |dvad| %.3g, band rel %.3g, %d segments, streams with moved bounds "
          "(stream, samples): %s" % (wv, wb, n_seg, diffs))


@pytest.mark.timeout(600)
@pytest.mark.parametrize("mode", ["staged", "fp16"])
def test_configs3_shard_512_streams(fvad_mod, oracle_mod, model, mode):
    """configs[3]'s per-GPU shard (4096 streams / 8 GPUs): 512 stereo streams
    of rank 3 (ids 1536..2047, so 26 digital-silence streams), 12 pushes of 50
    ticks with device VADMachines -- the persistent kernels' per-XCD queues,
    k_plpc's balanced grid and the recurrence kernels' workgroup counts at that
    size."""
    got, segs = run_engine(fvad_mod, model, mode, *SHARD)
    assert (got["vad"][500:600, 3::20] == 0).sum() > 1000  # ids 1539, 1559, ... = 19 mod 20
    ref = oracle_workload(*SHARD)
    if mode == "staged":
        n_seg = check_exact(ref, got, segs)
        print("configs[3] shard staged: 512 streams bit-exact, %d segments" % n_seg)
    else:
        wv, wb, n_seg, diffs = check_tolerance(ref, got, segs)
        print("configs[3] shard fp16: max |dvad| %.3g, band rel %.3g, %d segments, moved bounds %s" % (
            wv, wb, n_seg, diffs))


# bench.py:387-401: warmup pushes, a sync (the drain: k_vadm_par), the timed
# pushes back to back, a sync
SCHEDULES = {"bench": (5, 20), "nosync": (25, 0)}


def run_schedule(eng, schedule, log, n_streams):
    """The resident cycle from push 0 with the bench's schedule; the outputs of
    every push from the device log (log=True) or only the last push's (fetch)."""
    eng.reset()
    eng.resident_seek(0)
    n_pushes = sum(SCHEDULES[schedule])
    eng.output_log(n_pushes if log else 0)
    for n in SCHEDULES[schedule]:
        for _ in range(n):
            eng.run_resident(T)  # no sync in between: the host queues pushes ahead of the GPU
        if n:
            eng.sync()
    outs = [eng.output_log_read(k) for k in range(n_pushes)] if log else [eng.fetch(T)]
    got = {k: np.concatenate([o[k] for o in outs]) for k in outs[0]}
    segs = [eng.segments(s) for s in range(n_streams)]
    return got, segs, device_state(eng, n_streams)


def last_push(ref, n_ticks):
    """The oracle's outputs of the workload's last push only (fetch after the run)."""
    out = []
    for fr, wi, rsegs, st in ref:
        t0 = len(fr) - n_ticks
        wsel = wi["index"] + 2048 > fr["index"][t0]  # windows whose last sample is in the push
        out.append((fr[t0:], wi[wsel], rsegs, st))
    return out


@pytest.mark.timeout(1200)
def test_bench_schedule_staged_every_stream(fvad_mod, oracle_mod, model):
    """The bench's timed schedule itself: 2048 streams, the 25
    pushes of bench.py's default --warmup 5 --steps 20 through run_resident
    with no synchronisation between the pushes of a leg -- k_prep3 of push k+1
    beside push k (double-buffered xs / ratio / ticks), k_vadm_hbm of push k
    beside push k+1 on the side stream reading window-output set k & 1 in
    place, k_vadm_par only for the push before a sync.  Schedules: the bench's
    (5, sync, 20, sync) and 25 back to back.  Checked against the oracle fed
    the same 25 pushes: every stream's segments, VADMachine state and
    RollingAverage buffers after an unlogged run (the exact bench schedule),
    and every push's per-tick outputs from a run with the device output log.
    Then the same with every machine on k_vadm_par (FVAD_DEBUG_VADM_ALWAYS_PAR)
    and every third stream forced through k_vadm_par's in-kernel serial
    fallback (FVAD_DEBUG_VADM_PAR_SERIAL_EVERY = 3)."""
    base, B, P, R = BENCH
    eng = fvad_mod.Engine(model, B, 2, max_ticks=T, mode="staged")
    eng.attach_vadm()
    eng.load_synthetic(T, base=base, pushes=P)
    ref = oracle_workload(*BENCH)
    for schedule in ("bench", "nosync"):
        eng.set_debug(fvad_mod.DEBUG_VADM_COUNT, 1)
        got, segs, state = run_schedule(eng, schedule, False, B)
        cnt = eng.debug_counts()
        eng.set_debug(fvad_mod.DEBUG_VADM_COUNT, 0)
        check_exact(last_push(ref, T), got, segs)
        check_state(ref, state)
        # how the lazy long-term walk decided its tests
        print("bench schedule %s: long-term tests %s" % (schedule, cnt))
        got, segs, state = run_schedule(eng, schedule, True, B)
        assert got["vad"].shape == (len(ref[0][0]), B)
        n_seg = check_exact(ref, got, segs)
        check_state(ref, state)
        print("bench schedule %s: 2048 streams x 25 pushes bit-exact, %d segments" % (schedule, n_seg))
    eng.set_debug(fvad_mod.DEBUG_VADM_ALWAYS_PAR, 1)
    eng.set_debug(fvad_mod.DEBUG_VADM_PAR_SERIAL_EVERY, 3)
    got, segs, state = run_schedule(eng, "nosync", True, B)
    check_exact(ref, got, segs)
    check_state(ref, state)
    print("k_vadm_par on every push, every third stream on its serial fallback: bit-exact")
    # the lazy walk with its bound made infinite: every test the estimate
    # would settle takes vadm_stream's open branch (the exact fold)
    eng.set_debug(fvad_mod.DEBUG_VADM_ALWAYS_PAR, 0)
    eng.set_debug(fvad_mod.DEBUG_VADM_PAR_SERIAL_EVERY, 0)
    eng.set_debug(fvad_mod.DEBUG_VADM_BOUND_SCALE, -1)
    eng.set_debug(fvad_mod.DEBUG_VADM_COUNT, 1)
    got, segs, state = run_schedule(eng, "nosync", True, B)
    cnt = eng.debug_counts()
    check_exact(ref, got, segs)
    check_state(ref, state)
    assert cnt["open"] > 0 and cnt["settled"] == 0, cnt
    print("bound made infinite: bit-exact, long-term tests %s" % cnt)


@pytest.mark.timeout(900)
def test_bench_schedule_fp16_every_stream(fvad_mod, oracle_mod, model):
    """The fp16 variant (configs[4]; bench.py's `variants.fp16` line) under the
    bench's own schedule: 2048 streams, the 25 pushes through
    run_resident with no synchronisation inside a leg -- k_prep3 of push k+1
    and k_vadm_hbm of push k beside push k+1's kernels -- every push's outputs
    from the device output log and every stream's segments, within
    check_tolerance's bounds and MAX_MOVED, for the bench's (5, sync, 20, sync)
    schedule and 25 back to back."""
    base, B, P, R = BENCH
    eng = fvad_mod.Engine(model, B, 2, max_ticks=T, mode="fp16")
    eng.attach_vadm()
    eng.load_synthetic(T, base=base, pushes=P)
    ref = oracle_workload(*BENCH)
    for schedule in ("bench", "nosync"):
        got, segs, _ = run_schedule(eng, schedule, True, B)
        assert got["vad"].shape == (len(ref[0][0]), B)
        wv, wb, n_seg, diffs = check_tolerance(ref, got, segs)
        print("fp16 bench schedule %s: max |dvad| %.3g, band rel %.3g, %d segments, moved bounds %s" % (
            schedule, wv, wb, n_seg, diffs))


@pytest.mark.timeout(900)
def test_bench_schedule_fused16_equals_fp16(fvad_mod, model):
    """configs[4]'s fused FFT -> feature -> GRU kernel (mode fp16_fused,
    k_fused16) at the bench's size and unsynchronised schedule: every push's
    outputs and every stream's segments IDENTICAL to the fp16 mode's (the same
    pitch-spectrum and GRU expressions, so not a tolerance check)."""
    base, B, P, R = BENCH
    res = {}
    for mode in ("fp16", "fp16_fused"):
        eng = fvad_mod.Engine(model, B, 2, max_ticks=T, mode=mode)
        eng.attach_vadm()
        eng.load_synthetic(T, base=base, pushes=P)
        res[mode] = run_schedule(eng, "nosync", True, B)[:2]
        del eng
    (ga, sa), (gb, sb) = res["fp16"], res["fp16_fused"]
    for key in ga:
        assert np.array_equal(ga[key], gb[key]), key
    assert sa == sb


@pytest.mark.timeout(600)
def test_bench_size_i16_equals_float(fvad_mod, model):
    """The 16-bit ingest at the bench's size (2048 stereo streams, 50-tick
    pushes, the host legs' engine with device VADMachines): k_prep3 reads the
    16-bit samples itself (no float copy), and every output and segment equals
    a float submit of k / 32768.0f, push for push, with three pushes in flight
    on both engines; ragged ticks on the last push."""
    B, P = 2048, 6
    src = fvad_mod.synth_ticks(0, B, 2, P * T, 0, P * T)
    q = np.clip(np.round(src * np.float32(32768.0)), -32768, 32767).astype(np.int16)
    qf = q.astype(np.float32) / np.float32(32768.0)
    valid = np.full(B, T, np.int32)
    valid[::7] = 13
    outs = []
    for kind in ("float", "i16"):
        eng = fvad_mod.Engine(model, B, 2, max_ticks=T, mode="staged")
        eng.attach_vadm()
        got, inflight = [], 0
        for k in range(P):
            if inflight == 3:
                got.append(eng.collect())
                inflight -= 1
            tv = valid if k == P - 1 else None
            if kind == "float":
                eng.submit(qf[k * T:(k + 1) * T], ticks_valid=tv)
            else:
                eng.submit_i16(q[k * T:(k + 1) * T], ticks_valid=tv)
            inflight += 1
        while inflight:
            got.append(eng.collect())
            inflight -= 1
        eng.sync()
        outs.append((got, [eng.segments(s) for s in range(B)]))
        del eng
    (fa, fs), (ia, is_) = outs
    for a, b in zip(fa, ia):
        for key in ("vad", "ratio", "win_flag", "win_ratio", "win_vad"):
            assert np.array_equal(a[key], b[key]), key
        wf = a["win_flag"].astype(bool)
        assert np.array_equal(a["band"][wf], b["band"][wf])
    assert fs == is_
