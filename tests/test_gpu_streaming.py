"""Streaming ingest (fvad_engine_input_slot / submit / collect) and the bench
configuration at full size, against the CPU oracle.

The simulator reads the next chunk while the pipeline processes the last one
(SimulationInstance.zig:194-203); here two pushes are in flight, the H2D copy
of push k+1 overlapping push k's kernels.  Outputs must be bit-identical to
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


@pytest.mark.parametrize("mode", ["staged", "fused"])
def test_submit_collect_equals_push(fvad_mod, models, mode):
    """Two pushes in flight, alternating caller buffers and the zero-copy input
    slot, ragged ticks: every output equals the synchronous push's."""
    m, _ = models
    secs = [6.0, 4.31, 5.5, 1.2, 6.0]
    streams = [fvad_mod.synth_stream(i, int(48000 * s), 2)[0] for i, s in zip((3, 19, 39, 8, 77), secs)]
    pushes = _chunks(streams, 40)
    ref_eng = fvad_mod.Engine(m, len(streams), 2, max_ticks=40, want_denoised=True, mode=mode)
    ref = [ref_eng.push(p, ticks_valid=v, denoised=True) for p, v in pushes]
    eng = fvad_mod.Engine(m, len(streams), 2, max_ticks=40, want_denoised=True, mode=mode)
    got, in_flight = [], 0
    for k, (p, v) in enumerate(pushes):
        if in_flight == 2:
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


def test_submit_limits(fvad_mod, models):
    m, _ = models
    eng = fvad_mod.Engine(m, 2, 2, max_ticks=8)
    with pytest.raises(fvad_mod.FvadError):
        eng.collect()  # nothing submitted
    z = np.zeros((8, 2, 2, FRAME), np.float32)
    eng.submit(z)
    eng.submit(z)
    with pytest.raises(fvad_mod.FvadError):
        eng.submit(z)  # two uncollected pushes in flight
    eng.collect(want=False)
    eng.submit(z)
    eng.collect(want=False)
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


def test_full_size_bench_config_parity(fvad_mod, oracle_mod, models):
    """The bench's exact engine (2048 stereo streams, 50-tick pushes, staged,
    device VADMachine attached): two resident pushes of the same 0.5 s (what
    bench.py times), then two streamed pushes (submit / collect) of t = 5..6 s,
    where every 20th stream is digital silence.  Every stream's vad, ratio,
    window flag / ratio / vad, band sums and segments equal the oracle's."""
    m, om = models
    B, T = 2048, 50
    n = T * FRAME
    eng = fvad_mod.Engine(m, B, 2, max_ticks=T)
    eng.attach_vadm()
    eng.load_synthetic(T, base=0)
    outs = []
    for _ in range(2):
        eng.run_resident(T)
        eng.sync()
        outs.append(eng.fetch(T))
    late = np.zeros((2, T, B, 2, FRAME), np.float32)
    xs = []
    for s in range(B):
        x0 = fvad_mod.synth_stream(s, n, 2)[0]  # what load_synthetic generated (the generator depends on the length)
        x = fvad_mod.synth_stream(s, 6 * 48000, 2)[0]
        xs.append(np.concatenate([x0, x0, x[:, 5 * 48000:6 * 48000]], axis=1))
        late[:, :, s] = x[:, 5 * 48000:6 * 48000].reshape(2, 2, T, FRAME).transpose(1, 2, 0, 3)
    eng.submit(late[0])
    eng.submit(late[1])
    outs.append(eng.collect())
    outs.append(eng.collect())
    eng.sync()
    got = {k: np.concatenate([o[k] for o in outs]) for k in outs[0]}
    assert (got["vad"][100:, 19::20] == 0).sum() > 1000  # the silent streams hit the E < 0.04 gate
    oracle_mod.tables()
    pushes = [(0, n), (n, 2 * n), (2 * n, 3 * n), (3 * n, 4 * n)]
    with cf.ThreadPoolExecutor(max_workers=16) as ex:
        ref = list(ex.map(_oracle_trace, [(x, pushes, om) for x in xs]))
    for s, (fr, wi, segs) in enumerate(ref):
        assert np.array_equal(fr["vad"], got["vad"][:, s]), (s, pu.first_mismatch(fr["vad"], got["vad"][:, s]))
        assert np.array_equal(fr["ratio"], got["ratio"][:, s]), s
        wf = got["win_flag"][:, s].astype(bool)
        assert len(wi) == wf.sum(), s
        assert np.array_equal(wi["band"][:, :2], got["band"][wf, s, :, 0]), s
        assert np.array_equal(wi["ratio"], got["win_ratio"][wf, s]), s
        assert np.array_equal(wi["vad"], got["win_vad"][wf, s]), s
        assert eng.segments(s) == segs, s
