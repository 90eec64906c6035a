"""BASELINE.json configs[4]'s variant: engine mode "fp16" (FVAD_MODE_FP16) runs
the GRU stack on the matrix cores (k_gru16: int8 weights as exact f16, f16
inputs, f32 accumulation) and is compared with the CPU oracle at the stated
tolerance of SURVEY.md 8(c), not bit for bit:

  per-frame vad          |d| <= 2e-2 (absolute)
  denoised PCM           rel-RMS <= DEN_RELRMS per stream
  band sums (FFT B)      |d| / max|band| <= BAND_REL per stream
  volume ratios          bit-identical (computed before the GRU)
  segments / Evaluator   identical, or the differences listed and bounded

Everything before the GRU (HP filter, FFT A, pitch analysis, features) is the
bit-exact staged pipeline, so only the gains, vad and what depends on them can
differ.
"""
import concurrent.futures as cf

import numpy as np
import pytest

import parity_util as pu

pytestmark = pytest.mark.gpu

# SURVEY.md 8(c) states vad |d| <= 2e-2 for this config; measured on the
# synthetic set (tools/fp16_diag.py): max |dvad| 6.6e-5, denoised rel-RMS
# 1.7e-4, band rel 3.0e-4 -- the tests hold the tighter bounds below so a
# regression shows long before the stated tolerance is reached
VAD_ABS = 1e-3
DEN_RELRMS = 2e-3
BAND_REL = 2e-3


@pytest.fixture(scope="module")
def models(fvad_mod, oracle_mod):
    return fvad_mod.Model(seed=1), oracle_mod.Model(seed=1)


def check_stream(ref, got, ch, tag):
    fr = ref["frames"]
    assert len(fr) == len(got["vad"]), tag
    dv = float(np.abs(fr["vad"] - got["vad"]).max()) if len(fr) else 0.0
    assert dv <= VAD_ABS, (tag, dv)
    assert np.array_equal(fr["ratio"], got["ratio"]), tag
    dr, dg = ref["denoised"], got["denoised"]
    rel = float(np.sqrt(np.mean((dr - dg) ** 2)) / max(1e-12, np.sqrt(np.mean(dr ** 2))))
    assert rel <= DEN_RELRMS, (tag, rel)
    wi = ref["windows"]
    assert len(wi) == int(got["win_flag"].sum()), tag
    assert np.array_equal(wi["ratio"], got["win_ratio"]), tag
    b_ref, b_got = wi["band"][:, :ch], got["band"][:, :, 0]
    brel = float(np.abs(b_ref - b_got).max() / max(1e-12, np.abs(b_ref).max())) if len(wi) else 0.0
    assert brel <= BAND_REL, (tag, brel)
    return dv, rel, brel


def test_fp16_ragged_vs_oracle(fvad_mod, oracle_mod, models):
    """Ragged stereo streams (digital silence included: stream 19) in ragged
    pushes, the same cases the bit-exact modes pass exactly."""
    m, om = models
    secs = [12.0, 9.99, 7.0, 2.5]
    ids = [0, 1, 19, 42]
    streams = [fvad_mod.synth_stream(i, int(48000 * s), 2)[0] for i, s in zip(ids, secs)]
    ref = pu.oracle_run(oracle_mod, om, streams)
    eng = fvad_mod.Engine(m, len(streams), 2, max_ticks=37, want_denoised=True, mode="fp16")
    got = pu.engine_run(fvad_mod, eng, streams, 37)
    worst = [check_stream(r, g, 2, i) for r, g, i in zip(ref, got, ids)]
    print("fp16 ragged: max |dvad| %.3g, denoised rel-RMS %.3g, band rel %.3g" %
          tuple(max(w[k] for w in worst) for k in range(3)))


@pytest.mark.parametrize("n_channels", [1, 3])
def test_fp16_channels(fvad_mod, oracle_mod, models, n_channels):
    m, om = models
    streams = [fvad_mod.synth_stream(i, 48000 * 6, n_channels)[0] for i in (5, 6)]
    ref = pu.oracle_run(oracle_mod, om, streams)
    eng = fvad_mod.Engine(m, 2, n_channels, max_ticks=50, want_denoised=True, mode="fp16")
    got = pu.engine_run(fvad_mod, eng, streams, 50)
    for r, g, s in zip(ref, got, (5, 6)):
        check_stream(r, g, n_channels, s)


def test_fp16_many_streams_partial_workgroups(fvad_mod, oracle_mod, models):
    """37 streams (2 full 16-stream workgroups + 5), ragged lengths: every
    MFMA column maps to its own stream."""
    m, om = models
    ids = list(range(100, 137))
    secs = [3.0 + 0.07 * (i % 11) for i in range(len(ids))]
    streams = [fvad_mod.synth_stream(i, int(48000 * s), 2)[0] for i, s in zip(ids, secs)]
    oracle_mod.tables()
    with cf.ThreadPoolExecutor(max_workers=16) as ex:
        ref = list(ex.map(lambda x: pu.oracle_run(oracle_mod, om, [x])[0], streams))
    eng = fvad_mod.Engine(m, len(streams), 2, max_ticks=64, want_denoised=True, mode="fp16")
    got = pu.engine_run(fvad_mod, eng, streams, 64)
    for r, g, i in zip(ref, got, ids):
        check_stream(r, g, 2, i)


def _oracle_segments(args):
    import oracle
    import fvad
    sid, secs = args
    x, lab = fvad.synth_stream(sid, int(48000 * secs), 2)
    p = oracle.Pipeline(2, oracle.Model(seed=1))
    for k in range(0, x.shape[1], 48000):
        p.push([x[0, k:k + 48000], x[1, k:k + 48000]])
    return p.segments(), lab


def test_fp16_twenty_streams_evaluator(fvad_mod, oracle_mod, models):
    """configs[2]'s labelled set (20 stereo streams x 120 s) through the fp16
    engine with device VADMachines: segment lists are compared with the oracle's
    and every difference is reported; Evaluator TP/FP/FN (simulator.zig:123-128
    settings).  Measured: identical segment lists and TP/FP/FN."""
    m, _ = models
    secs, ids, T = 120.0, list(range(20)), 100
    streams = [fvad_mod.synth_stream(i, int(48000 * secs), 2)[0] for i in ids]
    eng = fvad_mod.Engine(m, len(ids), 2, max_ticks=T, mode="fp16")
    eng.attach_vadm()
    n = streams[0].shape[1] // 480
    for t0 in range(0, n, T):
        nt = min(T, n - t0)
        pcm = np.stack([x[:, t0 * 480:(t0 + nt) * 480].reshape(2, nt, 480).transpose(1, 0, 2) for x in streams], 1)
        eng.push(pcm)
    oracle_mod.tables()
    with cf.ThreadPoolExecutor(max_workers=10) as ex:
        ref = list(ex.map(_oracle_segments, [(i, secs) for i in ids]))
    to_sec = lambda segs: [(a / 48000.0, b / 48000.0) for a, b, _, _ in segs]
    cfg = dict(ignore_shorter_than_sec=0.7, extrude_start=5, extrude_end=10, fill_gaps=5)
    same, diffs, tot = 0, [], {"g": [0.0, 0.0, 0.0], "o": [0.0, 0.0, 0.0], "pos": 0.0}
    for s, (ref_segs, labels) in enumerate(ref):
        got = eng.segments(s)
        a = [(x[0], x[1]) for x in got]
        b = [(x[0], x[1]) for x in ref_segs]
        if a == b:
            same += 1
        else:
            diffs.append((s, sorted(set(a) ^ set(b))))
        sg = fvad_mod.evaluate(to_sec(got), labels, **cfg)
        so = oracle_mod.evaluate(to_sec(ref_segs), labels, **cfg)
        for i, k in enumerate(("true_positives_sec", "false_positives_sec", "false_negatives_sec")):
            tot["g"][i] += sg[k]
            tot["o"][i] += so[k]
        tot["pos"] += so["total_positives_sec"]
    print("fp16 20 x 120 s: %d/20 streams with identical segment bounds; differing bounds: %s" % (same, diffs))
    print("fp16 TP/FP/FN s: %s vs oracle %s (labelled %.1f s)" % (tot["g"], tot["o"], tot["pos"]))
    # measured: all 20 segment lists identical and TP/FP/FN equal to the oracle's
    assert same == 20, diffs
    assert tot["g"] == tot["o"], tot


def test_fp16_fft_size_1000_segments(fvad_mod, oracle_mod, models):
    """fp16 mode with a non-default VAD.Config (fft_size 1000: FFT B on the
    mixed-radix block kernel, bands from FFT.freqToBin) and device VADMachines:
    vad within tolerance, volume ratios and window ratios bit-identical (they
    come before the GRU), band sums within BAND_REL, segment lists identical
    to the oracle's (measured)."""
    m, om = models
    fft_size = 1000
    step = np.float32(48000) / np.float32(fft_size)
    bins = tuple(int(np.floor(np.float32(f) / step + np.float32(0.5))) for f in (100.0, 1500.0))
    ids, secs = (0, 19), (20.0, 13.3)
    streams = [fvad_mod.synth_stream(i, int(48000 * s), 2)[0] for i, s in zip(ids, secs)]
    eng = fvad_mod.Engine(m, len(streams), 2, max_ticks=50, fft_size=fft_size, bands=(bins,), mode="fp16")
    eng.attach_vadm()
    got = pu.engine_run(fvad_mod, eng, streams, 50, denoised=False)
    for s, x in enumerate(streams):
        n = x.shape[1]
        p = oracle_mod.Pipeline(2, om, fft_size=fft_size, trace_frames=n // 480 + 1,
                                trace_windows=n // fft_size + 2)
        for k in range(0, n, 48000):
            p.push([x[0, k:k + 48000], x[1, k:k + 48000]])
        fr, wi = p.trace()
        g = got[s]
        assert float(np.abs(fr["vad"] - g["vad"]).max()) <= VAD_ABS
        assert np.array_equal(fr["ratio"], g["ratio"])
        assert len(wi) == int(g["win_flag"].sum()) > 0
        assert np.array_equal(wi["ratio"], g["win_ratio"])
        b_ref, b_got = wi["band"][:, :2], g["band"][:, :, 0]
        assert float(np.abs(b_ref - b_got).max() / np.abs(b_ref).max()) <= BAND_REL
        assert [(a, b) for a, b, _, _ in eng.segments(s)] == [(a, b) for a, b, _, _ in p.segments()]

