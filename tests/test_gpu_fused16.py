"""BASELINE.json configs[4]'s fused FFT -> feature -> GRU kernel: engine mode
"fp16_fused" (FVAD_MODE_FP16_FUSED) runs k_fused16, the pitch-spectrum FFT,
its features 34..40 and the fp16 GRU stack in one kernel, in place of
k_pspecw + k_gru16.  The FFT is k_pspecw's per-frame code (fvad_wavedev.h:
pspec_frame) and the GRU k_gru16's, so every output must be IDENTICAL to the
fp16 mode's -- bit for bit, not within a tolerance.  The fp16 mode itself is
held to SURVEY.md 8(c)'s tolerance against the oracle (test_gpu_fp16.py); one
oracle check here covers the fused mode directly.
"""
import numpy as np
import pytest

import parity_util as pu
from test_gpu_fp16 import check_stream

pytestmark = pytest.mark.gpu

KEYS = ("vad", "ratio", "win_flag", "win_ratio", "win_vad", "band", "denoised")


@pytest.fixture(scope="module")
def model(fvad_mod):
    return fvad_mod.Model(seed=1)


def _run(fvad_mod, model, streams, mode, chunk, ch):
    eng = fvad_mod.Engine(model, len(streams), ch, max_ticks=chunk, want_denoised=True, mode=mode)
    return pu.engine_run(fvad_mod, eng, streams, chunk)


def _same(a, b, tag):
    for s, (x, y) in enumerate(zip(a, b)):
        for k in KEYS:
            assert np.array_equal(x[k], y[k]), (tag, s, k)


@pytest.mark.parametrize("n_channels", [1, 2, 3, 8])
def test_fused16_equals_fp16_ragged(fvad_mod, model, n_channels):
    """Ragged streams (digital silence in stream 19), ragged pushes, 13
    streams: one full 8-stream workgroup and a partial one; up to the 8
    channels an engine takes (8 interleaved frames per tick and stream)."""
    ids = [0, 1, 19, 42, 5, 6, 7, 8, 9, 10, 11, 12, 13]
    secs = [7.0, 5.99, 6.5, 2.5] + [3.0 + 0.11 * i for i in range(9)]
    streams = [fvad_mod.synth_stream(i, int(48000 * s), n_channels)[0] for i, s in zip(ids, secs)]
    a = _run(fvad_mod, model, streams, "fp16", 37, n_channels)
    b = _run(fvad_mod, model, streams, "fp16_fused", 37, n_channels)
    _same(a, b, n_channels)


def test_fused16_short_pushes(fvad_mod, model):
    """Pushes of 1 and 2 ticks: the prologue's two frames and a superstep loop
    shorter than its pipeline depth."""
    streams = [fvad_mod.synth_stream(i, 48000 * 2, 2)[0] for i in (3, 4, 19)]
    for chunk in (1, 2):
        a = _run(fvad_mod, model, streams, "fp16", chunk, 2)
        b = _run(fvad_mod, model, streams, "fp16_fused", chunk, 2)
        _same(a, b, chunk)


def test_fused16_vs_oracle(fvad_mod, oracle_mod, model):
    """The fused mode against the CPU oracle at configs[4]'s tolerance."""
    om = oracle_mod.Model(seed=1)
    ids, secs = [0, 19, 42], [9.99, 7.0, 4.0]
    streams = [fvad_mod.synth_stream(i, int(48000 * s), 2)[0] for i, s in zip(ids, secs)]
    ref = pu.oracle_run(oracle_mod, om, streams)
    got = _run(fvad_mod, model, streams, "fp16_fused", 50, 2)
    for r, g, i in zip(ref, got, ids):
        check_stream(r, g, 2, i)


def test_fused16_kernel_names(fvad_mod, model):
    """The fused engine launches k_fused16 in k_gru16's slot and no k_pspecw."""
    streams = [fvad_mod.synth_stream(i, 48000, 2)[0] for i in (0, 1)]
    eng = fvad_mod.Engine(model, 2, 2, max_ticks=50, mode="fp16_fused")
    pu.engine_run(fvad_mod, eng, streams, 50, denoised=False)
    kt = eng.kernel_times()["kernels"]
    assert "k_fused16" in kt and "k_gru16" not in kt and "k_rnn3" not in kt, kt
