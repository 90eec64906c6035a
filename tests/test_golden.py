"""Golden fixtures (tests/golden/): the oracle must keep reproducing its
committed outputs (CPU), and the HIP engine must reproduce them bit-exactly
without the oracle in the loop (GPU).  Regenerate with
tests/golden/make_golden.py only when the restated algorithm changes."""
import hashlib
import json
import os

import numpy as np
import pytest

import parity_util as pu

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
META = json.load(open(os.path.join(HERE, "oracle_seed1.json")))
ARR = np.load(os.path.join(HERE, "oracle_seed1.npz"))
CASES = sorted(META["cases"])


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def golden(name):
    g = {k: ARR["%s__%s" % (name, k)] for k in ("vad", "ratio", "win_band", "win_ratio", "win_vad", "den_head")}
    g.update(META["cases"][name])
    return g


def inputs(fvad_mod, g):
    x, _ = fvad_mod.synth_stream(g["stream_id"], int(48000 * g["seconds"]), g["channels"])
    assert sha(x) == g["input_sha256"], "synthetic generator drifted"
    return x


def test_model_blob_matches_golden(fvad_mod, oracle_mod):
    assert sha(oracle_mod.Model(seed=META["model_seed"]).blob()) == META["model_blob_sha256"]
    assert sha(fvad_mod.Model(seed=META["model_seed"]).blob()) == META["model_blob_sha256"]


@pytest.mark.parametrize("name", CASES)
def test_oracle_reproduces_golden(fvad_mod, oracle_mod, name):
    g = golden(name)
    x = inputs(fvad_mod, g)
    ref = pu.oracle_run(oracle_mod, oracle_mod.Model(seed=META["model_seed"]), [x])[0]
    fr, wi = ref["frames"], ref["windows"]
    assert np.array_equal(fr["vad"], g["vad"]) and np.array_equal(fr["ratio"], g["ratio"])
    assert np.array_equal(wi["band"][:, :g["channels"]], g["win_band"])
    assert np.array_equal(wi["ratio"], g["win_ratio"]) and np.array_equal(wi["vad"], g["win_vad"])
    assert sha(ref["denoised"].astype(np.float32)) == g["den_sha256"]
    assert [[int(a), int(b)] for a, b, _, _ in ref["segments"]] == g["segments"]


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["staged", "fused"])
def test_engine_reproduces_golden(fvad_mod, mode):
    m = fvad_mod.Model(seed=META["model_seed"])
    for name in CASES:
        g = golden(name)
        x = inputs(fvad_mod, g)
        eng = fvad_mod.Engine(m, 1, g["channels"], max_ticks=64, want_denoised=True, mode=mode)
        got = pu.engine_run(fvad_mod, eng, [x], 64)[0]
        assert np.array_equal(got["vad"], g["vad"]), (name, pu.first_mismatch(got["vad"], g["vad"]))
        assert np.array_equal(got["ratio"], g["ratio"]), name
        assert np.array_equal(got["band"][:, :, 0], g["win_band"]), name
        assert np.array_equal(got["win_ratio"], g["win_ratio"]) and np.array_equal(got["win_vad"], g["win_vad"])
        assert np.array_equal(got["denoised"][:, :960], g["den_head"]), name
        assert sha(got["denoised"].astype(np.float32)) == g["den_sha256"], name


@pytest.mark.gpu
def test_pipeline_segments_match_golden(fvad_mod):
    m = fvad_mod.Model(seed=META["model_seed"])
    for name in CASES:
        g = golden(name)
        x = inputs(fvad_mod, g)
        p = fvad_mod.AudioPipeline(m, g["channels"])
        p.push_samples([x[c] for c in range(g["channels"])])
        assert [[int(a), int(b)] for a, b, *_ in p.segments()] == g["segments"], name
