"""VAD.Config beyond the defaults on the device path, bit-exact against the
oracle: any even fft_size (FFT.zig:28-31; kissfft mixed radix on the GPU) --
below 480 one denoiser frame fills several FFT buffers (VAD.zig:307-347), above
16384 FFT B works in device scratch -- and use_denoiser = false (VAD.zig:206-212,239-249: fft_size frames of raw input
straight to FFT B, window ratio = preAnalyzeSegment over the frame, no vad).
"""
import numpy as np
import pytest

import parity_util as pu

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def models(fvad_mod, oracle_mod):
    return fvad_mod.Model(seed=1), oracle_mod.Model(seed=1)


def speech_bins(fft_size):
    """FFT.freqToBin (FFT.zig:120-131) of VADMachine's default 100..1500 Hz, f32."""
    step = np.float32(48000) / np.float32(fft_size)
    return tuple(int(np.floor(np.float32(f) / step + np.float32(0.5))) for f in (100.0, 1500.0))


def oracle_windows(oracle_mod, om, x, fft_size, use_denoiser, chunk, main_cfg=None):
    Ch, n = x.shape
    p = oracle_mod.Pipeline(Ch, om, fft_size=fft_size, use_denoiser=use_denoiser, main_cfg=main_cfg,
                            trace_frames=n // 480 + 1, trace_windows=n // fft_size + 2)
    for k in range(0, n, chunk):
        p.push([x[c, k:k + chunk] for c in range(Ch)])
    fr, wi = p.trace()
    return fr, wi, p.segments()


def engine_windows(fvad_mod, eng, streams, T):
    per = pu.engine_run(fvad_mod, eng, streams, T, denoised=False)
    return per


@pytest.mark.parametrize("fft_size", [480, 1000, 1024, 3000, 2 * 1009, 4096, 8192])
def test_engine_fft_sizes(fvad_mod, oracle_mod, models, fft_size):
    """Stereo streams through the staged engine at non-default FFT sizes
    (radices 4, 2, 3, 5 and a generic prime): per-frame vad / ratio and every
    window's band sums, ratio and vad equal the oracle's; device VADMachine
    segments equal the oracle's."""
    m, om = models
    secs = [20.0, 13.3]
    streams = [fvad_mod.synth_stream(i, int(48000 * s), 2)[0] for i, s in zip((0, 19), secs)]
    bins = speech_bins(fft_size)
    eng = fvad_mod.Engine(m, len(streams), 2, max_ticks=50, fft_size=fft_size, bands=(bins,))
    eng.attach_vadm()
    got = engine_windows(fvad_mod, eng, streams, 50)
    for s, x in enumerate(streams):
        fr, wi, segs = oracle_windows(oracle_mod, om, x, fft_size, True, 48000)
        g = got[s]
        assert np.array_equal(fr["vad"], g["vad"]) and np.array_equal(fr["ratio"], g["ratio"])
        assert len(wi) == int(g["win_flag"].sum()) > 0
        assert np.array_equal(wi["band"][:, :2], g["band"][:, :, 0])
        assert np.array_equal(wi["ratio"], g["win_ratio"]) and np.array_equal(wi["vad"], g["win_vad"])
        assert eng.segments(s) == segs


@pytest.mark.parametrize("fft_size", [2048, 1000, 4096])
def test_engine_without_denoiser(fvad_mod, oracle_mod, models, fft_size):
    """use_denoiser = false: windows are the raw input in fft_size frames; band
    sums, window ratios and segments equal the oracle's (window vad -1)."""
    m, om = models
    secs = [45.0, 31.9, 12.0]
    streams = [fvad_mod.synth_stream(i, int(48000 * s), 2)[0] for i, s in zip((3, 19, 4), secs)]
    bins = speech_bins(fft_size)
    eng = fvad_mod.Engine(m, len(streams), 2, max_ticks=64, fft_size=fft_size, bands=(bins,), use_denoiser=False,
                          want_denoised=True)
    eng.attach_vadm()
    got = pu.engine_run(fvad_mod, eng, streams, 64, denoised=True)
    n_segs = 0
    for s, x in enumerate(streams):
        _, wi, segs = oracle_windows(oracle_mod, om, x, fft_size, False, 48000)
        g = got[s]
        assert (g["vad"] == -1).all() and (g["ratio"] == -1).all()
        n = g["denoised"].shape[1]
        assert np.array_equal(g["denoised"], x[:, :n])  # the input passes through
        assert len(wi) == int(g["win_flag"].sum()) > 0
        assert np.array_equal(wi["band"][:, :2], g["band"][:, :, 0])
        assert np.array_equal(wi["ratio"], g["win_ratio"])
        assert (wi["vad"] == -1).all() and (g["win_vad"] == -1).all()
        assert eng.segments(s) == segs
        n_segs += len(segs)
    if fft_size == 2048:
        assert n_segs > 0


def test_fused_mode_size_limits(fvad_mod, models):
    m, _ = models
    with pytest.raises(fvad_mod.FvadError):
        fvad_mod.Engine(m, 1, 2, fft_size=2 * 1009, mode="fused")  # generic radix: staged only
    with pytest.raises(fvad_mod.FvadError):
        fvad_mod.Engine(m, 1, 2, fft_size=4096, mode="fused")
    with pytest.raises(fvad_mod.FvadError):
        fvad_mod.Engine(m, 1, 2, use_denoiser=False, mode="fused")
    with pytest.raises(fvad_mod.FvadError):
        fvad_mod.Engine(m, 1, 2, fft_size=256, mode="fused")  # < 480: the staged engine's window slots
    with pytest.raises(fvad_mod.FvadError):
        fvad_mod.Engine(m, 1, 2, fft_size=1001)  # odd (FFT.zig:29-31)
    with pytest.raises(fvad_mod.FvadError):
        fvad_mod.Engine(m, 1, 2, fft_size=0, bands=((0, 0),))
    with pytest.raises(fvad_mod.FvadError):
        fvad_mod.Engine(m, 1, 2, fft_size=1 << 23)  # beyond kMaxFftSize (32-bit window indices)


def test_without_denoiser_partial_ticks_engine(fvad_mod, oracle_mod, models):
    """use_denoiser = false counts samples, not ticks (VAD.zig:206-220 reads
    fft_size frames): a stream's last tick may be partial (last_tick_samples)
    and a window whose last sample sits in it still completes.  Stream lengths
    2048, 3 * 2048 and 5 s + 7 samples: 1, 3 and every window of the oracle,
    bit for bit."""
    m, om = models
    lens = [2048, 3 * 2048, 48000 * 5 + 7]
    streams = [fvad_mod.synth_stream(i, n, 2)[0] for i, n in zip((3, 19, 4), lens)]
    eng = fvad_mod.Engine(m, len(streams), 2, max_ticks=64, bands=(speech_bins(2048),), use_denoiser=False)
    T = max((n + 479) // 480 for n in lens)
    wins = [[] for _ in streams]
    for t0 in range(0, T, 64):
        nt = min(64, T - t0)
        pcm = np.zeros((nt, len(streams), 2, 480), np.float32)
        valid = np.zeros(len(streams), np.int32)
        last = np.full(len(streams), 480, np.int32)
        for s, x in enumerate(streams):
            a, b = t0 * 480, min(x.shape[1], (t0 + nt) * 480)
            if b <= a:
                continue
            k = b - a
            valid[s] = (k + 479) // 480
            last[s] = k - (valid[s] - 1) * 480
            seg = np.zeros((2, valid[s] * 480), np.float32)
            seg[:, :k] = x[:, a:b]
            pcm[:valid[s], s] = seg.reshape(2, valid[s], 480).transpose(1, 0, 2)
        o = eng.push(pcm, ticks_valid=valid, last_tick_samples=last)
        for s in range(len(streams)):
            wf = o["win_flag"][:valid[s], s].astype(bool)
            wins[s].append((o["band"][:valid[s], s][wf, :, 0], o["win_ratio"][:valid[s], s][wf]))
    for s, x in enumerate(streams):
        _, wi, _ = oracle_windows(oracle_mod, om, x, 2048, False, 48000)
        band = np.concatenate([b for b, _ in wins[s]])
        ratio = np.concatenate([r for _, r in wins[s]])
        assert len(wi) == len(band) == x.shape[1] // 2048, s
        assert np.array_equal(wi["band"][:, :2], band), s
        assert np.array_equal(wi["ratio"], ratio), s


def test_without_denoiser_pipeline_odd_pushes(fvad_mod, oracle_mod, models):
    """AudioPipeline (use_denoiser = false) fed odd-sized pushes: after EVERY
    push its segments equal the oracle's after the same push (a window is
    taken as soon as its samples are in, never a tick later)."""
    m, om = models
    x = fvad_mod.synth_stream(21, 48000 * 40 + 333, 2)[0]
    pipe = fvad_mod.AudioPipeline(m, 2, use_denoiser=False)
    ref = oracle_mod.Pipeline(2, om, fft_size=2048, use_denoiser=False)
    rng = np.random.default_rng(5)
    pos, n_checks, n_segs = 0, 0, 0
    while pos < x.shape[1]:
        k = int(min(x.shape[1] - pos, rng.integers(1, 40000)))
        pipe.push_samples([x[0, pos:pos + k], x[1, pos:pos + k]])
        ref.push([x[0, pos:pos + k], x[1, pos:pos + k]])
        pos += k
        assert pipe.segments() == ref.segments(), pos
        n_checks += 1
        n_segs = len(ref.segments())
    assert n_checks > 10 and n_segs > 0


def test_without_denoiser_multi_ragged_tails(fvad_mod, oracle_mod, models):
    """fvad_multi (the simulator core) with use_denoiser = false and stream
    lengths that end inside a tick: the final partial tick is submitted, so the
    segments equal the oracle's, the last window included."""
    m, om = models
    lens = [48000 * 30 + 2048 + 100, 48000 * 22 + 4095, 48000 * 31 + 1]
    ids = (3, 19, 8)
    streams = [fvad_mod.synth_stream(i, n, 2)[0] for i, n in zip(ids, lens)]
    multi = fvad_mod.Multi(m, len(streams), 2, devices=(0,), ticks_per_push=50, use_denoiser=False)
    multi.run_stream(streams, chunk=4801)
    for s, x in enumerate(streams):
        _, _, segs = oracle_windows(oracle_mod, om, x, 2048, False, 48000)
        assert multi.segments(s) == segs, s


def test_partial_tick_needs_no_denoiser(fvad_mod, models):
    """With the denoiser a 480-sample frame is never cut (VAD.zig:219)."""
    m, _ = models
    eng = fvad_mod.Engine(m, 1, 2, max_ticks=4)
    with pytest.raises(fvad_mod.FvadError):
        eng.push(np.zeros((2, 1, 2, 480), np.float32), last_tick_samples=[100])
    eng.push(np.zeros((2, 1, 2, 480), np.float32), last_tick_samples=[480])  # full ticks: fine


def windows_per_tick(fft_size):
    return 1 if fft_size >= 480 else (fft_size - 1 + 480) // fft_size


# stream lengths (s) per size.  fft_size 2 completes 24 000 windows per
# second, and every window re-sums the whole long-term average
# (RollingAverage.zig:45-56: the default initial value makes all 180 s of
# entries count from the start, 4.3 M at fft_size 2), so that case is short and
# its machine averages 0.2 s
SMALL_SECS = {2: (0.6, 0.37), 64: (12.0, 7.3), 256: (20.0, 13.3), 478: (20.0, 13.3)}


def machine_cfgs(fvad_mod, oracle_mod, fft_size):
    cf, co = fvad_mod.VadmConfig.default(), oracle_mod.VadmConfig.default()
    if fft_size == 2:
        cf.long_term_speech_avg_sec = co.long_term_speech_avg_sec = 0.2
    return cf, co


@pytest.mark.parametrize("fft_size", [2, 64, 256, 478])
def test_engine_small_fft_sizes(fvad_mod, oracle_mod, models, fft_size):
    """fft_size < 480 (VAD.zig:307-347): a 480-sample denoiser frame is split
    over several FFT-buffer writes, each piece adding ratio * written /
    fft_size; every full buffer is a window whose vad is the frame's.  The
    engine reports them in windows_per_tick slots per tick; per-frame vad /
    ratio, every window's band sums, ratio and vad, and the device
    VADMachine's segments equal the oracle's."""
    m, om = models
    streams = [fvad_mod.synth_stream(i, int(48000 * s), 2)[0] for i, s in zip((0, 19), SMALL_SECS[fft_size])]
    eng = fvad_mod.Engine(m, len(streams), 2, max_ticks=50, fft_size=fft_size, bands=(speech_bins(fft_size),))
    assert eng.wpt == windows_per_tick(fft_size)
    cf, co = machine_cfgs(fvad_mod, oracle_mod, fft_size)
    eng.attach_vadm([cf])
    got = engine_windows(fvad_mod, eng, streams, 50)
    for s, x in enumerate(streams):
        fr, wi, segs = oracle_windows(oracle_mod, om, x, fft_size, True, 48000, co)
        g = got[s]
        assert np.array_equal(fr["vad"], g["vad"]) and np.array_equal(fr["ratio"], g["ratio"])
        assert len(wi) == int(g["win_flag"].sum()) == (x.shape[1] // 480 * 480) // fft_size
        assert g["win_flag"].max() <= eng.wpt
        assert np.array_equal(wi["band"][:, :2], g["band"][:, :, 0])
        assert np.array_equal(wi["ratio"], g["win_ratio"]) and np.array_equal(wi["vad"], g["win_vad"])
        assert eng.segments(s) == segs


def run_partial_ticks(fvad_mod, eng, streams, chunk):
    """Push streams of any length (the last tick partial: last_tick_samples,
    use_denoiser = 0) in chunk-tick pushes; per stream the completed windows'
    band sums [n][C] and ratios, in order."""
    B, Ch = len(streams), streams[0].shape[0]
    lens = [x.shape[1] for x in streams]
    T = max((n + 479) // 480 for n in lens)
    bands = [[] for _ in streams]
    ratios = [[] for _ in streams]
    for t0 in range(0, T, chunk):
        nt = min(chunk, T - t0)
        pcm = np.zeros((nt, B, Ch, 480), np.float32)
        valid = np.zeros(B, np.int32)
        last = np.full(B, 480, np.int32)
        for s, x in enumerate(streams):
            a, b = t0 * 480, min(x.shape[1], (t0 + nt) * 480)
            if b <= a:
                continue
            k = b - a
            valid[s] = (k + 479) // 480
            last[s] = k - (valid[s] - 1) * 480
            seg = np.zeros((Ch, valid[s] * 480), np.float32)
            seg[:, :k] = x[:, a:b]
            pcm[:valid[s], s] = seg.reshape(Ch, valid[s], 480).transpose(1, 0, 2)
        o = eng.push(pcm, ticks_valid=valid, last_tick_samples=last)
        for s in range(B):
            cnt = o["win_flag"][:valid[s], s]
            bands[s].append(pu.tick_windows(o["band"][:valid[s], s], cnt, eng.wpt)[:, :, 0])
            ratios[s].append(pu.tick_windows(o["win_ratio"][:valid[s], s], cnt, eng.wpt))
    return [np.concatenate(b) for b in bands], [np.concatenate(r) for r in ratios]


@pytest.mark.parametrize("fft_size", [2, 64, 256, 478])
def test_engine_small_fft_without_denoiser(fvad_mod, oracle_mod, models, fft_size):
    """use_denoiser = false with fft_size < 480: the pipeline reads fft_size
    frames (VAD.zig:206-220), so one 480-sample tick holds several windows;
    stream ends mid-tick (last_tick_samples).  Band sums and window ratios of
    every window equal the oracle's; the device VADMachine's segments too."""
    m, om = models
    secs = SMALL_SECS[fft_size]
    lens = [int(48000 * secs[0]) + 7, int(48000 * secs[1]) + 333]
    streams = [fvad_mod.synth_stream(i, n, 2)[0] for i, n in zip((3, 19), lens)]
    eng = fvad_mod.Engine(m, len(streams), 2, max_ticks=40, fft_size=fft_size, bands=(speech_bins(fft_size),),
                          use_denoiser=False)
    cf, co = machine_cfgs(fvad_mod, oracle_mod, fft_size)
    eng.attach_vadm([cf])
    band, ratio = run_partial_ticks(fvad_mod, eng, streams, 40)
    for s, x in enumerate(streams):
        _, wi, segs = oracle_windows(oracle_mod, om, x, fft_size, False, 48000, co)
        assert len(wi) == len(band[s]) == x.shape[1] // fft_size
        assert np.array_equal(wi["band"][:, :2], band[s])
        assert np.array_equal(wi["ratio"], ratio[s])
        assert eng.segments(s) == segs


@pytest.mark.parametrize("fft_size,use_denoiser", [(20480, True), (22528, True), (22528, False)])
def test_engine_large_fft_sizes(fvad_mod, oracle_mod, models, fft_size, use_denoiser):
    """fft_size > 16384: FFT B's tables outside the plan and the transform in
    device scratch (20480 = 2 * 4^5 * 2 * 5; 22528 = 2 * 4^5 * 11, a generic
    radix).  Band sums, ratios, vad and the device VADMachine's segments equal
    the oracle's.  (Up to 24000: above it VADMachine.init's channel-ratio
    average has length 0, VADMachine.zig:73,89-93.)"""
    m, om = models
    streams = [fvad_mod.synth_stream(i, int(48000 * s), 2)[0] for i, s in zip((0, 19), (16.0, 11.3))]
    eng = fvad_mod.Engine(m, len(streams), 2, max_ticks=50, fft_size=fft_size, bands=(speech_bins(fft_size),),
                          use_denoiser=use_denoiser)
    eng.attach_vadm()
    got = engine_windows(fvad_mod, eng, streams, 50)
    for s, x in enumerate(streams):
        fr, wi, segs = oracle_windows(oracle_mod, om, x, fft_size, use_denoiser, 48000)
        g = got[s]
        if use_denoiser:
            assert np.array_equal(fr["vad"], g["vad"]) and np.array_equal(fr["ratio"], g["ratio"])
        assert len(wi) == int(g["win_flag"].sum()) > 0
        assert np.array_equal(wi["band"][:, :2], g["band"][:, :, 0])
        assert np.array_equal(wi["ratio"], g["win_ratio"])
        if use_denoiser:
            assert np.array_equal(wi["vad"], g["win_vad"])
        assert eng.segments(s) == segs


def test_engine_fft_65536(fvad_mod, oracle_mod, models):
    """fft_size 65536 (4^7 * 2 complex points, 512 KB of scratch per
    transform), with a VADMachine whose channel-ratio average spans 2 s: the
    reference's default 0.5 s gives that average length 0 above fft_size 24000
    (VADMachine.zig:73,89-93).  Window outputs and segments equal the
    oracle's."""
    m, om = models
    x = fvad_mod.synth_stream(4, 48000 * 9, 2)[0]
    fft = 65536
    cfg_f, cfg_o = fvad_mod.VadmConfig.default(), oracle_mod.VadmConfig.default()
    cfg_f.channel_vol_ratio_avg_sec = cfg_o.channel_vol_ratio_avg_sec = 2.0
    eng = fvad_mod.Engine(m, 1, 2, max_ticks=64, fft_size=fft, bands=(speech_bins(fft), (0, 4000)))
    eng.attach_vadm([cfg_f])
    got = engine_windows(fvad_mod, eng, [x], 64)[0]
    p = oracle_mod.Pipeline(2, om, fft_size=fft, main_cfg=cfg_o, trace_frames=901, trace_windows=8)
    p.push([x[0], x[1]])
    fr, wi = p.trace()
    assert np.array_equal(fr["vad"], got["vad"])
    assert len(wi) == int(got["win_flag"].sum()) == 6
    assert np.array_equal(wi["band"][:, :2], got["band"][:, :, 0])
    assert np.array_equal(wi["ratio"], got["win_ratio"]) and np.array_equal(wi["vad"], got["win_vad"])
    assert eng.segments(0) == p.segments()
