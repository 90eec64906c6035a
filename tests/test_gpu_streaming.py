"""Streaming ingest (fvad_engine_input_slot / submit / collect) and the bench
configuration at full size, against the CPU oracle.

The simulator reads the next chunk while the pipeline processes the last one
(SimulationInstance.zig:194-203); here up to three pushes are in flight, the
H2D copy of push k+2 overlapping push k+1's kernels.  Outputs must be bit-identical to
the synchronous push and to the oracle.
"""
import concurrent.futures as cf

import numpy as np
import pytest

import parity_util as pu

pytestmark = pytest.mark.gpu

FRAME = 480


@pytest.fixture(scope="module")
def models(fvad_mod, oracle_mod):
    return fvad_mod.Model(seed=1), oracle_mod.Model(seed=1)


def _chunks(streams, nt_push):
    """[ticks][streams][ch][480] pushes with ragged ticks_valid, as engine_run builds them."""
    B, Ch = len(streams), streams[0].shape[0]
    lens = [x.shape[1] // FRAME for x in streams]
    out = []
    for t0 in range(0, max(lens), nt_push):
        nt = min(nt_push, max(lens) - t0)
        pcm = np.zeros((nt, B, Ch, FRAME), np.float32)
        valid = np.zeros(B, np.int32)
        for s, x in enumerate(streams):
            v = max(0, min(nt, lens[s] - t0))
            valid[s] = v
            if v:
                pcm[:v, s] = x[:, t0 * FRAME:(t0 + v) * FRAME].reshape(Ch, v, FRAME).transpose(1, 0, 2)
        out.append((pcm, valid))
    return out


@pytest.mark.parametrize("mode,depth", [("staged", 2), ("fused", 2), ("staged", 3), ("fp16", 3), ("fp16_fused", 3)])
def test_submit_collect_equals_push(fvad_mod, models, mode, depth):
    """depth (2 or FVAD_MAX_IN_FLIGHT = 3) pushes in flight, alternating caller
    buffers and the zero-copy input slot, ragged ticks: every output equals
    the synchronous push's."""
    m, _ = models
    secs = [6.0, 4.31, 5.5, 1.2, 6.0]
    streams = [fvad_mod.synth_stream(i, int(48000 * s), 2)[0] for i, s in zip((3, 19, 39, 8, 77), secs)]
    pushes = _chunks(streams, 40)
    ref_eng = fvad_mod.Engine(m, len(streams), 2, max_ticks=40, want_denoised=True, mode=mode)
    ref = [ref_eng.push(p, ticks_valid=v, denoised=True) for p, v in pushes]
    eng = fvad_mod.Engine(m, len(streams), 2, max_ticks=40, want_denoised=True, mode=mode)
    got, in_flight = [], 0
    for k, (p, v) in enumerate(pushes):
        if in_flight == depth:
            got.append(eng.collect(denoised=True))
            in_flight -= 1
        if k % 2:
            slot = eng.input_slot()
            slot[: p.shape[0]] = p
            eng.submit(slot[: p.shape[0]], ticks_valid=v)
        else:
            eng.submit(p, ticks_valid=v)
        in_flight += 1
    while in_flight:
        got.append(eng.collect(denoised=True))
        in_flight -= 1
    assert len(got) == len(ref)
    for a, b in zip(ref, got):
        for key in ("vad", "ratio", "win_flag", "win_ratio", "win_vad", "denoised"):
            assert np.array_equal(a[key], b[key]), key
        wf = a["win_flag"].astype(bool)
        assert np.array_equal(a["band"][wf], b["band"][wf])


@pytest.mark.parametrize("mode,depth", [("staged", 3), ("fused", 2), ("fp16", 3), ("fp16_fused", 3)])
def test_submit_i16_equals_float_push(fvad_mod, models, mode, depth):
    """16-bit ingest (fvad_engine_submit_i16, k_pcm16): samples k give the
    outputs of a float push of k / 32768.0f (libsndfile's short -> float),
    bit for bit -- through the zero-copy 16-bit slot and caller buffers, depth
    pushes in flight, ragged ticks, full-scale and clipped samples."""
    m, _ = models
    secs = [5.0, 3.37, 4.2, 0.9]
    streams = []
    for i, sec in zip((5, 21, 44, 9), secs):
        x = fvad_mod.synth_stream(i, int(48000 * sec), 2)[0]
        q = np.clip(np.round(x * 32768.0 * (1 + 3 * (i == 44))), -32768, 32767).astype(np.int16)
        streams.append(q)
    q_pushes = _chunks([q.astype(np.float32) for q in streams], 30)  # sample values k, as f32
    ref_eng = fvad_mod.Engine(m, len(streams), 2, max_ticks=30, want_denoised=True, mode=mode)
    ref = [ref_eng.push(p / np.float32(32768.0), ticks_valid=v, denoised=True) for p, v in q_pushes]
    eng = fvad_mod.Engine(m, len(streams), 2, max_ticks=30, want_denoised=True, mode=mode)
    got, in_flight = [], 0
    for k, (p, v) in enumerate(q_pushes):
        p16 = p.astype(np.int16)
        if in_flight == depth:
            got.append(eng.collect(denoised=True))
            in_flight -= 1
        if k % 2:
            slot = eng.input_slot_i16()
            slot[: p16.shape[0]] = p16
            eng.submit_i16(slot[: p16.shape[0]], ticks_valid=v)
        else:
            eng.submit_i16(p16, ticks_valid=v)
        in_flight += 1
    while in_flight:
        got.append(eng.collect(denoised=True))
        in_flight -= 1
    assert len(got) == len(ref)
    for a, b in zip(ref, got):
        for key in ("vad", "ratio", "win_flag", "win_ratio", "win_vad", "denoised"):
            assert np.array_equal(a[key], b[key]), key
        wf = a["win_flag"].astype(bool)
        assert np.array_equal(a["band"][wf], b["band"][wf])


def test_submit_i16_no_denoiser_partial_tick(fvad_mod, models):
    """use_denoiser = 0 with a partial last tick through the 16-bit ingest."""
    m, _ = models
    n = [2048 * 3 + 100, 480 * 9 + 17]
    streams = [np.clip(np.round(fvad_mod.synth_stream(7 + i, k, 2)[0] * 32768.0), -32768, 32767).astype(np.int16)
               for i, k in enumerate(n)]
    T = max((k + FRAME - 1) // FRAME for k in n)
    pcm = np.zeros((T, 2, 2, FRAME), np.int16)
    valid = np.zeros(2, np.int32)
    last = np.zeros(2, np.int32)
    for s, x in enumerate(streams):
        nt = (x.shape[1] + FRAME - 1) // FRAME
        pad = np.zeros((2, nt * FRAME), np.int16)
        pad[:, : x.shape[1]] = x
        pcm[:nt, s] = pad.reshape(2, nt, FRAME).transpose(1, 0, 2)
        valid[s] = nt
        last[s] = x.shape[1] - (nt - 1) * FRAME
    ref_eng = fvad_mod.Engine(m, 2, 2, max_ticks=T, use_denoiser=False)
    ref = ref_eng.push(pcm.astype(np.float32) / np.float32(32768.0), ticks_valid=valid, last_tick_samples=last)
    eng = fvad_mod.Engine(m, 2, 2, max_ticks=T, use_denoiser=False)
    eng.submit_i16(pcm, ticks_valid=valid, last_tick_samples=last)
    got = eng.collect()
    n_win = 0
    for s in range(2):  # outputs are defined on each stream's valid ticks, windows where win_flag is set
        wf = ref["win_flag"][: valid[s], s].astype(bool)
        assert np.array_equal(wf, got["win_flag"][: valid[s], s].astype(bool)), s
        for key in ("win_ratio", "win_vad", "band"):
            assert np.array_equal(ref[key][: valid[s], s][wf], got[key][: valid[s], s][wf]), (key, s)
        n_win += int(wf.sum())
    assert n_win == sum(k // 2048 for k in n)


def test_submit_limits(fvad_mod, models):
    m, _ = models
    eng = fvad_mod.Engine(m, 2, 2, max_ticks=8)
    with pytest.raises(fvad_mod.FvadError):
        eng.collect()  # nothing submitted
    z = np.zeros((8, 2, 2, FRAME), np.float32)
    for _ in range(3):
        eng.submit(z)
    with pytest.raises(fvad_mod.FvadError):
        eng.submit(z)  # FVAD_MAX_IN_FLIGHT = 3 uncollected pushes in flight
    eng.collect(want=False)
    eng.submit(z)
    for _ in range(3):
        eng.collect(want=False)


def _oracle_trace(args):
    import oracle
    x, pushes, om = args
    Ch, n = x.shape
    frames = n // FRAME
    p = oracle.Pipeline(Ch, om, trace_frames=frames + 1, trace_windows=frames // 4 + 2)
    for a, b in pushes:
        p.push([x[c, a:b] for c in range(Ch)])
    fr, wi = p.trace()
    return fr, wi, p.segments()


def test_multi_two_partitions(fvad_mod, oracle_mod, models):
    """fvad_multi with two partitions (two engines on device 0, one host thread
    each, streaming submits): partition + merge give the oracle's segments."""
    m, om = models
    secs = [40.0, 31.7, 40.0, 12.3, 25.0, 40.0, 7.7]
    ids = [0, 1, 2, 19, 39, 5, 6]
    streams = [fvad_mod.synth_stream(i, int(48000 * s), 2)[0] for i, s in zip(ids, secs)]
    multi = fvad_mod.Multi(m, len(streams), 2, devices=(0, 0), ticks_per_push=64)
    multi.run(streams)
    oracle_mod.tables()
    with cf.ThreadPoolExecutor(max_workers=len(streams)) as ex:
        ref = list(ex.map(_oracle_trace, [(x, [(0, x.shape[1])], om) for x in streams]))
    n = 0
    for s, (_, _, segs) in enumerate(ref):
        assert multi.segments(s) == segs, s
        n += len(segs)
    assert n > 3


def test_multi_three_unequal_partitions(fvad_mod, oracle_mod, models):
    """fvad_multi over three partitions of unequal size on device 0 (8 streams
    -> parts of 2, 3, 3: one engine and host thread each, as the simulator's
    one-thread-per-instance runAll, simulator.zig:217-228), fed by the
    streaming reader in 48 000-frame reads: every stream's segments equal the
    oracle's, whichever part it landed in."""
    m, om = models
    secs = [30.0, 21.7, 30.0, 9.3, 25.0, 30.0, 14.4, 27.9]
    ids = [0, 1, 2, 19, 39, 5, 59, 7]
    streams = [fvad_mod.synth_stream(i, int(48000 * s), 2)[0] for i, s in zip(ids, secs)]
    multi = fvad_mod.Multi(m, len(streams), 2, devices=(0, 0, 0), ticks_per_push=50)
    multi.run_stream(streams)
    oracle_mod.tables()
    with cf.ThreadPoolExecutor(max_workers=len(streams)) as ex:
        ref = list(ex.map(_oracle_trace, [(x, [(0, x.shape[1])], om) for x in streams]))
    n = 0
    for s, (_, _, segs) in enumerate(ref):
        assert multi.segments(s) == segs, s
        n += len(segs)
    assert n > 3
