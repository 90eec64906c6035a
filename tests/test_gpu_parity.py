"""Parity of the HIP hot path (through the C ABI) with the CPU oracle.

Contract: the kernels reproduce the oracle's arithmetic
operation-for-operation (-ffp-contract=off, correctly rounded f32 div/sqrt, C
promotion rules), so every output is compared for BIT EQUALITY.  The stated
fall-back tolerances of the north star (per-frame vad |d| <= 1e-4, denoised
rel-RMS <= 1e-5, band sums rel <= 1e-5, identical segments and TP/FP/FN) are
therefore met with zero margin used.
"""
import concurrent.futures as cf

import numpy as np
import pytest

import parity_util as pu

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def models(fvad_mod, oracle_mod):
    return fvad_mod.Model(seed=1), oracle_mod.Model(seed=1)


def assert_stream_equal(ref, got, ch):
    fr = ref["frames"]
    assert len(fr) == len(got["vad"])
    assert np.array_equal(fr["vad"], got["vad"]), pu.first_mismatch(fr["vad"], got["vad"])
    assert np.array_equal(fr["ratio"], got["ratio"]), pu.first_mismatch(fr["ratio"], got["ratio"])
    if ref["denoised"] is not None:
        assert np.array_equal(ref["denoised"], got["denoised"]), pu.first_mismatch(ref["denoised"], got["denoised"])
    wi = ref["windows"]
    assert len(wi) == int(got["win_flag"].sum())
    assert np.array_equal(wi["band"][:, :ch], got["band"][:, :, 0])
    assert np.array_equal(wi["ratio"], got["win_ratio"])
    assert np.array_equal(wi["vad"], got["win_vad"])


@pytest.mark.parametrize("mode", ["staged", "fused"])
def test_engine_bit_exact_ragged(fvad_mod, oracle_mod, models, mode):
    """Stereo streams of different (non-multiple-of-480) lengths, pushed in
    ragged chunks: every per-frame and per-window output is bit-identical."""
    m, om = models
    secs = [12.0, 9.99, 7.0, 2.5]
    ids = [0, 1, 19, 42]
    streams = [fvad_mod.synth_stream(i, int(48000 * s), 2)[0] for i, s in zip(ids, secs)]
    ref = pu.oracle_run(oracle_mod, om, streams)
    eng = fvad_mod.Engine(m, len(streams), 2, max_ticks=37, want_denoised=True, mode=mode)
    got = pu.engine_run(fvad_mod, eng, streams, 37)
    for r, g in zip(ref, got):
        assert_stream_equal(r, g, 2)


def periodic_streams(n):
    """Strictly periodic inputs: their pitch cross-correlations repeat at every
    multiple of the period, so the coarse and fine find_best_pitch scans see
    runs of (near-)equal xcorr^2 / Syy ratios -- the case the staged path's
    survivor filter (k_pcorr Q1) must get exactly right."""
    t = np.arange(n) / 48000.0
    sigs = [
        0.3 * np.sin(2 * np.pi * 200.0 * t),                      # period 240 samples
        0.25 * np.sign(np.sin(2 * np.pi * 150.0 * t)),            # square wave, period 320
        0.2 * ((np.arange(n) % 480) == 0).astype(np.float64),     # impulse train, period 480
        0.2 * (2 * ((np.arange(n) % 96) / 96.0) - 1),             # sawtooth, period 96 (x_lp: 48)
        0.1 * np.sin(2 * np.pi * 250.0 * t) + 0.1 * np.sin(2 * np.pi * 500.0 * t),
        np.full(n, 0.05),                                         # DC
    ]
    out = []
    for i in range(0, len(sigs), 2):
        out.append(np.stack([sigs[i], sigs[i + 1]]).astype(np.float32))
    return out


@pytest.mark.parametrize("mode", ["staged", "fused"])
def test_engine_periodic_inputs(fvad_mod, oracle_mod, models, mode):
    """Tones, a square wave, an impulse train, a sawtooth and DC (3 s stereo):
    every output bit-identical with the oracle."""
    m, om = models
    streams = periodic_streams(48000 * 3)
    ref = pu.oracle_run(oracle_mod, om, streams)
    eng = fvad_mod.Engine(m, len(streams), 2, max_ticks=50, want_denoised=True, mode=mode)
    got = pu.engine_run(fvad_mod, eng, streams, 50)
    for r, g in zip(ref, got):
        assert_stream_equal(r, g, 2)


@pytest.mark.parametrize("mode", ["staged", "fused"])
@pytest.mark.parametrize("n_channels,fft_size", [(1, 2048), (2, 512), (3, 2048)])
def test_engine_channels_and_fft_size(fvad_mod, oracle_mod, models, n_channels, fft_size, mode):
    m, om = models
    streams = [fvad_mod.synth_stream(i, 48000 * 6, n_channels)[0] for i in (5, 6)]
    ref = []
    for x in streams:
        frames = x.shape[1] // 480
        p = oracle_mod.Pipeline(n_channels, om, fft_size=fft_size, trace_frames=frames + 1,
                                trace_windows=frames + 1, trace_denoised=frames * 480)
        p.push([x[c] for c in range(n_channels)])
        fr, wi = p.trace()
        ref.append({"frames": fr, "windows": wi, "denoised": p.tden[:, :frames * 480].copy()})
    bins = (1, 16) if fft_size == 512 else (4, 64)
    eng = fvad_mod.Engine(m, 2, n_channels, max_ticks=50, fft_size=fft_size, bands=(bins,), want_denoised=True,
                          mode=mode)
    got = pu.engine_run(fvad_mod, eng, streams, 50)
    for r, g in zip(ref, got):
        assert_stream_equal(r, g, n_channels)


def test_staged_equals_fused_resident(fvad_mod, models):
    """Both engine modes on the same resident synthetic batch (256 stereo
    streams x 3 pushes of 40 ticks): every output bit-identical."""
    m, _ = models
    outs = []
    for mode in ("staged", "fused"):
        eng = fvad_mod.Engine(m, 256, 2, max_ticks=40, mode=mode)
        eng.load_synthetic(40, 7)
        res = []
        for _ in range(3):
            eng.run_resident(40)
            res.append(eng.fetch(40))
        outs.append(res)
    for a, b in zip(*outs):
        for k in ("vad", "ratio", "win_flag", "win_ratio", "win_vad"):
            assert np.array_equal(a[k], b[k]), (k, pu.first_mismatch(a[k], b[k]))
        wf = a["win_flag"].astype(bool)  # band sums are only written for completed windows
        assert wf.sum() > 0 and np.array_equal(a["band"][wf], b["band"][wf])


def test_engine_multiple_bands(fvad_mod, oracle_mod, models):
    m, om = models
    alt = oracle_mod.VadmConfig.default()
    alt.speech_min_freq, alt.speech_max_freq = 300.0, 3000.0
    x = fvad_mod.synth_stream(3, 48000 * 5, 2)[0]
    eng = fvad_mod.Engine(m, 1, 2, max_ticks=500, bands=((4, 64), (13, 128)))
    out = eng.push(x.reshape(2, -1, 480).transpose(1, 0, 2)[:, None])
    p = oracle_mod.Pipeline(2, om, main_cfg=alt, trace_windows=200)
    p.push([x[0], x[1]])
    _, wi = p.trace()
    flags = out["win_flag"][:, 0].astype(bool)
    assert np.array_equal(out["band"][flags, 0, :, 1], wi["band"][:, :2])


def test_inactive_ticks_do_not_touch_state(fvad_mod, oracle_mod, models):
    """A stream with ticks_valid = 0 for a push keeps its state untouched."""
    m, om = models
    x = fvad_mod.synth_stream(9, 48000 * 3, 2)[0]
    frames = x.reshape(2, -1, 480).transpose(1, 0, 2)  # [T][2][480]
    eng = fvad_mod.Engine(m, 2, 2, max_ticks=100, want_denoised=True)
    pad = np.zeros((50, 2, 2, 480), np.float32)
    pad[:, 0] = frames[:50]
    o1 = eng.push(pad, ticks_valid=[50, 0], denoised=True)
    pad2 = np.zeros((100, 2, 2, 480), np.float32)
    pad2[:100, 0] = frames[50:150]
    pad2[:, 1] = frames[:100]
    o2 = eng.push(pad2, ticks_valid=[100, 100], denoised=True)
    # stream 1 saw its first frames only in the second push: must equal stream 0's first 100 ticks
    assert np.array_equal(o2["vad"][:, 1], np.concatenate([o1["vad"][:, 0], o2["vad"][:50, 0]]))
    assert np.array_equal(o2["denoised"][:, 1], np.concatenate([o1["denoised"][:, 0], o2["denoised"][:50, 0]]))


def test_rnnoise_compat_shim(fvad_mod, oracle_mod, models):
    """rnnoise_create/process_frame/destroy over the C ABI == oracle, frame by frame."""
    m, om = models
    assert fvad_mod.Denoiser.get_frame_size() == 480
    x = fvad_mod.synth_stream(2, 480 * 120, 1)[0][0] * np.float32(32767)
    d = fvad_mod.Denoiser(m)
    o = oracle_mod.Denoiser(om)
    for i in range(120):
        f = x[i * 480:(i + 1) * 480]
        a, va = d.process_s16(f)
        b, vb = o.process(f)
        assert va == vb and np.array_equal(a, b), i
    with pytest.raises(ValueError):
        d.process_s16(np.zeros(479, np.float32))


# every even nfft (kissfft mixed radix: 4, 2, 3, 5 and generic primes), odd
# ncfft included (n = 6, 10, 2 * 1009), LDS and global-memory work arrays
@pytest.mark.parametrize("n", [2, 6, 8, 10, 14, 22, 32, 60, 128, 240, 480, 512, 1000, 1024, 2000, 2048, 2 * 1009,
                               3 * 2048, 4096, 8192, 2 * 7 * 7 * 11, 16384, 40000])
def test_kiss_fftr_compat_shim(fvad_mod, oracle_mod, n):
    rng = np.random.default_rng(n)
    x = rng.standard_normal(n).astype(np.float32)
    a = fvad_mod.kiss_fftr(x)
    b, _ = oracle_mod.kiss_fftr(x)
    assert np.array_equal(a.real.astype(np.float32), b.real.astype(np.float32))
    assert np.array_equal(a.imag.astype(np.float32), b.imag.astype(np.float32))
    if n >= 8:  # and it is a DFT (kissfft accuracy), not just the oracle's bits
        ref = np.fft.rfft(x.astype(np.float64))
        assert np.abs(a - ref).max() <= 1e-4 * np.abs(ref).max() * np.log2(n)


def test_audio_pipeline_segments(fvad_mod, oracle_mod, models):
    """AudioPipeline.pushSamples in irregular chunks (incl. a sub-frame tail)
    gives the oracle's segment lists for the main and an alternative machine."""
    m, om = models
    x = fvad_mod.synth_stream(0, 48000 * 45 + 333, 2)[0]
    alt_f = fvad_mod.VadmConfig.default()
    alt_f.speech_threshold_factor = 9.0
    alt_o = oracle_mod.VadmConfig.default()
    alt_o.speech_threshold_factor = 9.0
    pipe = fvad_mod.AudioPipeline(m, 2, alt_cfgs=(alt_f,))
    pos = 0
    rng = np.random.default_rng(0)
    while pos < x.shape[1]:
        n = int(rng.integers(1, 60000))
        first = pipe.push_samples([x[0, pos:pos + n], x[1, pos:pos + n]])
        assert first == pos
        pos += n
    p = oracle_mod.Pipeline(2, om, alt_cfgs=(alt_o,))
    p.push([x[0], x[1]])
    assert pipe.segments() == p.segments()
    assert pipe.segments(0) == p.segments(0)
    assert len(p.segments()) > 0


def _oracle_segments(args):
    import oracle
    sid, secs = args
    import fvad
    x, lab = fvad.synth_stream(sid, int(48000 * secs), 2)
    om = oracle.Model(seed=1)
    p = oracle.Pipeline(2, om)
    for k in range(0, x.shape[1], 48000):
        p.push([x[0, k:k + 48000], x[1, k:k + 48000]])
    return p.segments(), lab


def test_twenty_streams_evaluator_parity(fvad_mod, oracle_mod, models):
    """configs[2]: 20 concurrent stereo streams (120 s each) on one MI355X —
    segment lists and Evaluator TP/FP/FN identical to the CPU oracle."""
    m, _ = models
    secs = 120.0
    ids = list(range(20))
    streams = [fvad_mod.synth_stream(i, int(48000 * secs), 2)[0] for i in ids]
    multi = fvad_mod.Multi(m, len(ids), 2, devices=(0,), ticks_per_push=100)
    multi.run(streams)
    oracle_mod.tables()  # build the oracle's lazily initialised tables before threading
    with cf.ThreadPoolExecutor(max_workers=10) as ex:  # ctypes releases the GIL
        ref = list(ex.map(_oracle_segments, [(i, secs) for i in ids]))
    stats_g, stats_o = [], []
    n_segs = 0
    for s, (ref_segs, labels) in enumerate(ref):
        got = multi.segments(s)
        assert got == ref_segs, s
        n_segs += len(got)
        to_sec = lambda segs: [(a / 48000.0, b / 48000.0) for a, b, _, _ in segs]
        cfg = dict(ignore_shorter_than_sec=0.7, extrude_start=5, extrude_end=10, fill_gaps=5)  # simulator.zig:123-128
        stats_g.append(fvad_mod.evaluate(to_sec(got), labels, **cfg))
        stats_o.append(oracle_mod.evaluate(to_sec(ref_segs), labels, **cfg))
    assert n_segs > 20
    for a, b in zip(stats_g, stats_o):
        for k in ("true_positives_sec", "false_positives_sec", "false_negatives_sec"):
            assert a[k] == b[k]


def test_full_size_determinism_and_spot_parity(fvad_mod, oracle_mod, models):
    """configs[4] per-GPU size (2048 streams): two runs from reset are bit-identical
    (no atomics / races), and sampled streams match the oracle."""
    m, om = models
    B, T = 2048, 24
    eng = fvad_mod.Engine(m, B, 2, max_ticks=T, want_denoised=True)
    eng.load_synthetic(T, base=0)
    eng.run_resident(T)
    eng.sync()
    o1 = eng.fetch(T, denoised=True)
    eng.reset()
    eng.run_resident(T)
    eng.sync()
    o2 = eng.fetch(T, denoised=True)
    for k in o1:
        assert np.array_equal(o1[k], o2[k]), k
    for s in (0, 19, 777, 2047):
        x = fvad_mod.synth_stream(s, T * 480, 2)[0]
        p = oracle_mod.Pipeline(2, om, trace_frames=T + 1, trace_windows=T, trace_denoised=T * 480)
        p.push([x[0], x[1]])
        fr, wi = p.trace()
        assert np.array_equal(fr["vad"], o1["vad"][:, s])
        assert np.array_equal(p.tden[:, :T * 480], o1["denoised"][:, s].transpose(1, 0, 2).reshape(2, -1))
        flags = o1["win_flag"][:, s].astype(bool)
        assert np.array_equal(wi["band"][:, :2], o1["band"][flags, s, :, 0])


def test_engine_argument_errors(fvad_mod, models):
    m, _ = models
    with pytest.raises(fvad_mod.FvadError):
        fvad_mod.Engine(m, 1, 2, fft_size=1001)  # odd: FFT.zig:29-31
    e = fvad_mod.Engine(m, 2, 2, max_ticks=4)
    with pytest.raises(fvad_mod.FvadError):
        e.push(np.zeros((5, 2, 2, 480), np.float32))
    with pytest.raises(fvad_mod.FvadError):
        e.push(np.zeros((2, 2, 2, 480), np.float32), ticks_valid=[3, 1])
    out = e.push(np.zeros((0, 2, 2, 480), np.float32))
    assert out["vad"].shape == (0, 2)
