"""Recorder / segment capture: AudioPipeline.zig:134-195,
Recorder.zig:52-146.  The reference captures the raw pushed input of every
completed main-machine segment, from VADMachine.getOffsetRecordingStart(speech
start) to getOffsetRecordingEnd(speech end) -- exactly the segment's
sample_from / sample_to -- and keeps the channel with the lowest rmsVolume.
The oracle restates that (oracle.recordings); parity is bit-exact."""
import numpy as np
import pytest


@pytest.mark.parametrize("n_channels,n", [(1, 1), (2, 7), (2, 48000), (3, 4801), (4, 480001)])
def test_recording_channel_matches_oracle(fvad_mod, oracle_mod, n_channels, n):
    rng = np.random.default_rng(n_channels * 1000 + n)
    for trial in range(5):
        chans = [(rng.standard_normal(n) * rng.uniform(0.01, 1.0)).astype(np.float32) for _ in range(n_channels)]
        assert fvad_mod.recording_channel(chans) == oracle_mod.recording_channel(chans)


def test_recording_channel_ties_and_silence(fvad_mod, oracle_mod):
    a = np.linspace(-0.5, 0.5, 960, dtype=np.float32)
    # identical channels: the first one (strict < in findBestChannel)
    assert fvad_mod.recording_channel([a, a.copy(), a.copy()]) == 0
    # a silent channel wins
    z = np.zeros(960, np.float32)
    assert fvad_mod.recording_channel([a, z]) == 1 == oracle_mod.recording_channel([a, z])
    # sign does not matter, order does
    assert fvad_mod.recording_channel([-a, a]) == 0


def test_oracle_recordings_cut_segments(oracle_mod):
    rng = np.random.default_rng(3)
    x = [rng.standard_normal(200000).astype(np.float32) * s for s in (1.0, 0.25)]
    segs = [(1000, 50000, 0.0, 0.0), (90000, 190000, 0.0, 0.0)]
    rec = oracle_mod.recordings(x, segs)
    assert [r[0] for r in rec] == [1000, 90000]
    assert all(r[1] == 1 for r in rec)
    assert np.array_equal(rec[0][2], x[1][1000:50000]) and np.array_equal(rec[1][2], x[1][90000:190000])


@pytest.fixture(scope="module")
def models(fvad_mod, oracle_mod):
    return fvad_mod.Model(seed=1), oracle_mod.Model(seed=1)


@pytest.mark.gpu
def test_audio_pipeline_recordings(fvad_mod, oracle_mod, models):
    """AudioPipeline with on_recording attached, pushed in irregular chunks: one
    recording per completed main-machine segment, identical to the oracle's."""
    m, om = models
    x = fvad_mod.synth_stream(0, 48000 * 45 + 333, 2)[0]
    pipe = fvad_mod.AudioPipeline(m, 2)
    pipe.record()
    pos = 0
    rng = np.random.default_rng(1)
    while pos < x.shape[1]:
        n = int(rng.integers(1, 60000))
        pipe.push_samples([x[0, pos:pos + n], x[1, pos:pos + n]])
        pos += n
    p = oracle_mod.Pipeline(2, om)
    p.push([x[0], x[1]])
    segs = p.segments()
    assert len(segs) > 0 and pipe.segments() == segs
    exp = oracle_mod.recordings([x[0], x[1]], segs)
    got = pipe.recordings
    assert len(got) == len(exp)
    for (s0, c0, a0), (s1, c1, a1) in zip(got, exp):
        assert (s0, c0) == (s1, c1)
        assert np.array_equal(a0, a1)
