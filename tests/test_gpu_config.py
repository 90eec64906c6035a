"""VAD.Config beyond the defaults on the device path, bit-exact against the
oracle: any even fft_size (FFT.zig:28-31; kissfft mixed radix on the GPU) and
use_denoiser = false (VAD.zig:206-212,239-249: fft_size frames of raw input
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


def oracle_windows(oracle_mod, om, x, fft_size, use_denoiser, chunk):
    Ch, n = x.shape
    p = oracle_mod.Pipeline(Ch, om, fft_size=fft_size, use_denoiser=use_denoiser,
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
        fvad_mod.Engine(m, 1, 2, fft_size=256)  # < 480: more than one window per tick
    with pytest.raises(fvad_mod.FvadError):
        fvad_mod.Engine(m, 1, 2, fft_size=1001)  # odd (FFT.zig:29-31)
