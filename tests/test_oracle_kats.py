"""Pin the CPU oracle (tests' checker) against every known-answer vector the
reference's own tests hold, plus KATs derived from the reference semantics
(SURVEY.md §8(c)).  CPU only."""
import numpy as np
import pytest


# ---------------- reference unit tests, ported as expected values ----------------

import json
import os

REF = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "reference_vectors.json")))


def test_segment_writer_reference_vector(oracle_mod):
    """SegmentWriter.zig:124-175 — pack a {1}{2,3,4} split source into 10 samples."""
    import ctypes as C
    O = oracle_mod
    v = REF["segment_writer"]
    buf = np.zeros(v["buffer_len"], np.float32)

    class SW(C.Structure):
        _fields_ = [("buf", C.c_void_p), ("len", C.c_size_t), ("write_index", C.c_size_t), ("index", C.c_uint64)]

    w = SW(buf.ctypes.data, v["buffer_len"], 0, 0)
    first = np.array(v["first"], np.float32)
    second = np.array(v["second"], np.float32)
    for k, (off, expect) in enumerate(v["writes"]):
        got = O.lib().ora_segwriter_write(C.byref(w), O.fptr(first), len(first), O.fptr(second), len(second), off,
                                          -1)
        assert got == expect
        if k == 2:
            assert w.write_index == v["write_index_after_third"]
    assert buf.tolist() == v["final_buffer"]


def test_multi_ring_buffer_reference_vectors(oracle_mod):
    """MultiRingBuffer.zig:203-249 — eight wrap-around write cases on capacity 5."""
    import ctypes as C
    O = oracle_mod
    v = REF["multi_ring_buffer"]

    class Ring(C.Structure):
        _fields_ = [("buf", C.c_void_p), ("capacity", C.c_size_t), ("total_write_count", C.c_uint64)]

    pcm = np.zeros(v["capacity"], np.int32)
    r = Ring(pcm.ctypes.data, v["capacity"], 0)
    for st in v["steps"]:
        a = np.array(st["src"], np.int32)
        O.lib().ora_ring_write(C.byref(r), a.ctypes.data_as(C.POINTER(C.c_int32)), len(a), st["offset"], st["n"])
        assert pcm.tolist() == st["expect"]


@pytest.mark.parametrize("case", REF["calc_false_positive"]["cases"])
def test_calc_false_positive_reference_vectors(oracle_mod, case):
    """statistics.zig:286-360 — refs [2,3],[4,5], extrude 2/2, fill gaps 2."""
    v = REF["calc_false_positive"]
    fp = oracle_mod.calc_false_positive_sec(case["vad"][0], case["vad"][1], [tuple(r) for r in v["refs"]],
                                            extrude_start=v["extrude_start"], extrude_end=v["extrude_end"],
                                            fill_gaps=v["fill_gaps"])
    assert abs(fp - case["expect"]) < v["tolerance"]


# ---------------- derived KATs ----------------

def test_fft_a_matches_dft(oracle_mod):
    rng = np.random.default_rng(0)
    x = (rng.standard_normal(960) + 1j * rng.standard_normal(960)).astype(np.complex64)
    y = oracle_mod.fft960(x)
    ref = np.fft.fft(x.astype(np.complex128)) / 960  # opus_fft scales by 1/nfft
    assert np.abs(y - ref).max() / np.abs(ref).max() < 1e-6


def test_fft_b_matches_rfft(oracle_mod):
    rng = np.random.default_rng(1)
    for n in (8, 32, 512, 2048, 1024, 96):
        x = rng.standard_normal(n).astype(np.float32)
        y, _ = oracle_mod.kiss_fftr(x)
        ref = np.fft.rfft(x.astype(np.float64))
        assert np.abs(y - ref).max() / np.abs(ref).max() < 2e-6, n


def test_fftzig_bin_centred_sine(oracle_mod):
    """FFT.zig normalisation: a bin-centred sine of amplitude A at bin k0 has
    mag[k0] = A and mag[k0+-1] = A/2 under the periodic Hann window, so the
    4..64 band sum is 2A."""
    w = oracle_mod.hann_periodic(2048)
    assert abs(2048 / w.astype(np.float64).sum() - 2.0) < 1e-6
    n = np.arange(2048)
    for A, k0 in ((0.5, 16), (0.25, 40), (1.0, 5)):
        s = (A * np.cos(2 * np.pi * k0 * n / 2048)).astype(np.float32)
        m = oracle_mod.fftzig(s, w)
        assert abs(m[k0] - A) < 1e-5 * max(1, A)
        assert abs(m[k0 - 1] - A / 2) < 1e-5 and abs(m[k0 + 1] - A / 2) < 1e-5
        assert abs(m[4:65].sum() - 2 * A) < 1e-4


def test_fftzig_rejects_odd_size(oracle_mod):
    with pytest.raises(ValueError):
        oracle_mod.fftzig(np.zeros(7, np.float32), np.ones(7, np.float32))


def test_rms_volume(oracle_mod):
    x = np.full(480, 0.5, np.float32)
    assert oracle_mod.rms_volume(x) == pytest.approx(0.5, abs=1e-7)


def test_tables(oracle_mod):
    hw, dct, tt = oracle_mod.tables()
    # tansig table = tanh(0.04 i) to 6 decimals
    i = np.arange(201)
    assert np.abs(tt - np.round(np.tanh(0.04 * i), 6)).max() < 1e-6
    # orthonormal DCT-II (with the sqrt(2/22) output scale)
    d = dct.astype(np.float64) * np.sqrt(2.0 / 22)
    assert np.abs(d @ d.T - np.eye(22)).max() < 1e-6
    # power-complementary Vorbis window
    assert np.abs(hw.astype(np.float64) ** 2 + hw[::-1].astype(np.float64) ** 2 - 1).max() < 1e-6


def test_rnnoise_perfect_reconstruction(oracle_mod, fvad_mod):
    """Weight-free KAT: with unit gains and no pitch filter, analysis + synthesis
    reproduce the high-passed input delayed by one frame (FFT A + window + OLA)."""
    O = oracle_mod
    x, _ = fvad_mod.synth_stream(3, 48000, 1)
    x = (x[0] * np.float32(32767)).astype(np.float32)
    d = O.Denoiser(O.Model(seed=1))
    d.set_bypass(1)
    ys = np.concatenate([d.process(x[i * 480:(i + 1) * 480])[0] for i in range(100)])
    # biquad in double, as denoise.c
    m0 = np.float32(0)
    m1 = np.float32(0)
    hp = np.zeros(48000, np.float32)
    a0, a1 = float(np.float32(-1.99599)), float(np.float32(0.996))
    for i in range(48000):
        xi = x[i]
        yi = np.float32(xi + m0)
        m0 = np.float32(float(m1) + (-2.0 * float(xi) - a0 * float(yi)))
        m1 = np.float32(float(xi) - a1 * float(yi))
        hp[i] = yi
    err = np.abs(ys[480:] - hp[:-480])
    for k in range(2, 99):
        seg = slice(k * 480, (k + 1) * 480)
        assert err[seg].max() <= 2e-6 * max(1.0, np.abs(hp[seg]).max())


def test_rnnoise_silence_gate(oracle_mod):
    """All-zero input: E < 0.04 gate -> vad 0, output 0, features cleared."""
    O = oracle_mod
    d = O.Denoiser(O.Model(seed=1))
    for _ in range(5):
        out, vad = d.process(np.zeros(480, np.float32))
        assert vad == 0.0
        assert not np.any(out)
        _, _, silence, feats = d.debug()
        assert silence == 1 and not np.any(feats)


def test_synthetic_model_is_rnnoise_shaped(oracle_mod):
    b = oracle_mod.Model(seed=7).blob()
    assert len(b) == 87503  # rnnoise parameter count (42-24-24-48-96-22-1 topology)
    assert b.min() >= -64 and b.max() <= 64


def test_model_text_roundtrip(oracle_mod, tmp_path):
    """rnnoise text model format: write the synthetic model, read it back."""
    O = oracle_mod
    m = O.Model(seed=3)
    path = tmp_path / "model.txt"
    write_text_model(m.blob(), path)
    m2 = O.Model(path=str(path))
    assert np.array_equal(m.blob(), m2.blob())


LAYERS = [(42, 24, 0, False), (24, 24, 2, True), (90, 48, 2, True), (114, 96, 2, True), (96, 22, 1, False),
          (24, 1, 1, False)]


def write_text_model(blob, path):
    lines = ["rnnoise-nu model file version 1"]
    o = 0
    for nin, nout, act, gru in LAYERS:
        g = 3 if gru else 1
        sizes = [nin * nout * g] + ([nout * nout * 3] if gru else []) + [nout * g]
        lines.append("%d %d %d" % (nin, nout, act))
        for n in sizes:
            lines.append(" ".join(str(int(v)) for v in blob[o:o + n]))
            o += n
    path.write_text("\n".join(lines) + "\n")


def test_audacity_parse(oracle_mod):
    txt = "1.5\t2.25\tspeech\n\n3\t4\tx\nbad-line-without-tab\n5.5\t6.5\tlast"
    segs = oracle_mod.parse_audacity(txt)
    assert segs.tolist() == [[1.5, 2.25], [3.0, 4.0], [5.5, 6.5]]
    with pytest.raises(ValueError):
        oracle_mod.parse_audacity("1\tnot-a-number\tx")
