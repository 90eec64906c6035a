"""Product host-side logic vs the oracle, and the C-ABI surface — CPU only
(no compute call needs a GPU here)."""
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "formula-vad_amd")


def test_abi_exports_every_declared_symbol(fvad_mod):
    """libfvad.so loads and exports every function include/fvad.h declares."""
    hdr = open(os.path.join(ROOT, "include", "fvad.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    hdr = "\n".join(l for l in hdr.split("\n")
                    if not l.lstrip().startswith("#") and not (l.lstrip().startswith("typedef") and "(*" in l))
    names = set(re.findall(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*\([^;{]*\)\s*;", hdr))
    names -= {"sizeof"}
    assert len(names) >= 40
    L = fvad_mod.lib()
    missing = [n for n in sorted(names) if not hasattr(L, n)]
    assert not missing, missing
    bound = {s[0] for s in fvad_mod.SYMBOLS}
    assert names <= bound, sorted(names - bound)


def test_header_constants_match_binding(fvad_mod):
    """The engine modes and debug keys the binding passes are the header's
    values (FVAD_MODE_FP16_FUSED, r6, included)."""
    hdr = open(os.path.join(ROOT, "include", "fvad.h")).read()
    defs = dict((k, int(v)) for k, v in re.findall(r"#define\s+(FVAD_[A-Z0-9_]+)\s+(-?\d+)\b", hdr))
    for name in ("MODE_STAGED", "MODE_FUSED", "MODE_FP16", "MODE_FP16_FUSED"):
        assert getattr(fvad_mod, name) == defs["FVAD_" + name], name
    for name in ("DEBUG_VADM_PAR_SERIAL_EVERY", "DEBUG_VADM_ALWAYS_PAR", "DEBUG_VADM_LT_FULL", "DEBUG_VADM_DEFER_MAX",
                 "DEBUG_VADM_BOUND_SCALE", "DEBUG_VADM_COUNT", "DEBUG_VADM_NEGATE_AT"):
        assert getattr(fvad_mod, name) == defs["FVAD_" + name], name


@pytest.mark.parametrize("seed", [0, 1, 1234, 2 ** 40 + 7])
def test_synthetic_model_identical_to_oracle(fvad_mod, oracle_mod, seed):
    assert np.array_equal(fvad_mod.Model(seed=seed).blob(), oracle_mod.Model(seed=seed).blob())


def test_text_model_loader(fvad_mod, oracle_mod, tmp_path):
    from test_oracle_kats import write_text_model
    blob = oracle_mod.Model(seed=5).blob()
    p = tmp_path / "m.txt"
    write_text_model(blob, p)
    assert np.array_equal(fvad_mod.Model(path=str(p)).blob(), blob)
    bad = tmp_path / "bad.txt"
    bad.write_text("rnnoise-nu model file version 2\n")
    with pytest.raises(fvad_mod.FvadError):
        fvad_mod.Model(path=str(bad))


def test_synth_deterministic(fvad_mod):
    a, la = fvad_mod.synth_stream(7, 48000 * 3, 2)
    b, lb = fvad_mod.synth_stream(7, 48000 * 3, 2)
    c, _ = fvad_mod.synth_stream(8, 48000 * 3, 2)
    assert np.array_equal(a, b) and np.array_equal(la, lb)
    assert not np.array_equal(a, c)
    assert np.abs(a).max() <= 1.0
    s, _ = fvad_mod.synth_stream(19, 48000 * 7, 2)  # every 20th stream: 1 s of digital silence at 5 s
    assert not np.any(s[:, 5 * 48000:6 * 48000])


def random_segments(rng, n, t_max=120.0):
    starts = np.sort(rng.uniform(0, t_max, n))
    return [(float(s), float(s + rng.uniform(0.2, 8))) for s in starts]


@pytest.mark.parametrize("seed", range(6))
def test_evaluator_matches_oracle(fvad_mod, oracle_mod, seed):
    rng = np.random.default_rng(seed)
    vad = random_segments(rng, rng.integers(0, 25))
    ref = random_segments(rng, rng.integers(1, 25))
    for cfg in [dict(ignore_shorter_than_sec=0.7), dict(ignore_shorter_than_sec=0.7, extrude_start=5, extrude_end=10,
                                                         fill_gaps=5)]:
        a = fvad_mod.evaluate(vad, ref, **cfg)
        b = oracle_mod.evaluate(vad, ref, **cfg)
        for k in a:
            assert (np.isnan(a[k]) and np.isnan(b[k])) or a[k] == b[k], (k, a[k], b[k])


def test_aggregate_matches_oracle(fvad_mod, oracle_mod):
    rng = np.random.default_rng(11)
    stats = [oracle_mod.evaluate(random_segments(rng, 10), random_segments(rng, 10), 0.7, 5, 10, 5)
             for _ in range(5)]
    a = fvad_mod.aggregate(stats)
    b = oracle_mod.aggregate(stats)
    for name in ("total_positives_sec", "true_positives_sec", "false_positives_sec", "false_negatives_sec",
                 "fm_index", "f_score"):
        assert getattr(a, name) == getattr(b, name)
    for name in ("true_positive_rate", "false_negative_rate", "false_discovery_rate", "precision"):
        for f in ("overall", "min", "max", "avg"):
            assert getattr(getattr(a, name), f) == getattr(getattr(b, name), f)


def test_parse_audacity_matches_oracle(fvad_mod, oracle_mod):
    txt = "0.5\t1.75\tspeech\r\n2\t3\t\n\n4.125\t9.0\tx"
    assert np.array_equal(fvad_mod.parse_audacity(txt), oracle_mod.parse_audacity(txt))
    with pytest.raises(ValueError):
        fvad_mod.parse_audacity("1\t2\r\n")  # CR kept in the 'to' field (formats.zig:11-14)


def test_vadmachine_matches_oracle(fvad_mod, oracle_mod):
    """Product VADMachine fed the oracle's per-window band sums / ratio / vad
    reproduces the oracle's segment list exactly."""
    O = oracle_mod
    om = O.Model(seed=1)
    x, _ = fvad_mod.synth_stream(1, 48000 * 40, 2)
    p = O.Pipeline(2, om, trace_frames=5000, trace_windows=1000)
    p.push([x[0], x[1]])
    _, wins = p.trace()
    vm = fvad_mod.VADMachine(n_channels=2)
    assert vm.bins() == (4, 64)
    for w in wins:
        vm.run(int(w["index"]), w["band"][:2], float(w["vad"]), float(w["ratio"]))
    ref = p.segments()
    got = vm.segments()
    assert len(ref) > 0
    assert got == ref


def test_vadmachine_alt_config_bins(fvad_mod):
    c = fvad_mod.VadmConfig.default()
    c.speech_min_freq, c.speech_max_freq = 300.0, 3000.0
    assert fvad_mod.VADMachine(c).bins() == (13, 128)


def test_engine_fails_loudly_without_gpu(fvad_mod):
    from conftest import gpu_available
    if gpu_available():
        pytest.skip("GPU present")
    with pytest.raises(fvad_mod.FvadError):
        fvad_mod.Engine(fvad_mod.Model(seed=1), 2)


def test_instrumented_counts_match_cost_model(fvad_mod, oracle_mod):
    """fvad/cost.py MEASURED is what tests/count_ops.py counts on the bench
    input (fine-search lags, remove_doubling candidates, silent frames)."""
    import count_ops
    from fvad import cost
    got = count_ops.count(threads=8)
    for k, v in cost.MEASURED.items():
        assert got[k] == pytest.approx(v, abs=1e-4), k


def test_cpu_baseline_native_build_same_work(oracle_mod, fvad_mod):
    """The -O3 -march=native CPU-baseline flavour runs the same algorithm:
    identical work counts on the same input."""
    import numpy as np
    L, _ = oracle_mod.native_lib()
    pcm = np.stack([fvad_mod.synth_stream(s, 48000, 2)[0] for s in (0, 19)])
    _, a = oracle_mod.bench_pipeline(pcm, chunk=24000, n_threads=2)
    _, b = oracle_mod.bench_pipeline(pcm, chunk=24000, n_threads=2, L=L)
    assert a == b and a["frames"] == 2 * 100 * 2


@pytest.mark.parametrize("n", [2, 6, 1000, 1024, 2048, 2 * 1009, 40000])
def test_kiss_fftr_alloc_lenmem_protocol(fvad_mod, n):
    """FFT.zig:193-208 probes kiss_fftr_alloc(n, 0, NULL, &lenmem = 1): it must
    fail and write the size; FFT.zig:179-191 then builds the cfg in caller
    memory.  Host-only (no device call)."""
    import ctypes as C
    L = fvad_mod.lib()
    lenmem = C.c_size_t(1)
    assert L.kiss_fftr_alloc(n, 0, None, C.byref(lenmem)) is None
    assert lenmem.value > 0
    small = C.c_size_t(lenmem.value - 1)
    mem = C.create_string_buffer(lenmem.value)
    assert L.kiss_fftr_alloc(n, 0, mem, C.byref(small)) is None and small.value == lenmem.value
    got = C.c_size_t(lenmem.value)
    assert L.kiss_fftr_alloc(n, 0, mem, C.byref(got)) == C.addressof(mem)
    assert L.kiss_fftr_alloc(n + 1, 0, None, C.byref(C.c_size_t(1))) is None  # odd sizes refused


def test_synth_ticks_host_memory_bounded():
    """fvad_synth_ticks / fvad_engine_load_synthetic_ex keep no whole-block
    cache (a rank of an 8-GPU run held its 7.9 GB block): the
    peak RSS of a process that takes 50 ticks of 256 streams x 10 s (the
    generator runs the full length per stream) grows by the output plus the
    generator threads' per-stream scratch, not by the 0.98 GB block."""
    import subprocess
    import sys
    code = r'''
import resource, sys
sys.path.insert(0, %r)
import fvad
fvad.lib()
r0 = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss
x = fvad.synth_ticks(0, 256, 2, 1000, 0, 50)
y = fvad.synth_ticks(0, 256, 2, 1000, 950, 50)
r1 = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss
assert x.shape == (50, 256, 2, 480) and y.shape == x.shape and float(abs(x).max()) > 0
print((r1 - r0) / 1024.0)
''' % PKG
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    grew_mb = float(out.stdout.strip().splitlines()[-1])
    out_mb = 2 * 50 * 256 * 2 * 480 * 4 / 2 ** 20  # 93.75
    assert grew_mb < out_mb + 16 * 3.84 * 2 + 64, grew_mb  # < ~280 MB, against ~1 GB with a block cache


def test_add_const_n_exact(tmp_path):
    """fvad_exact.h's add_const_n (the long-term RollingAverage's recompute over
    entries still holding the initial average, RollingAverage.zig:45-56, per
    binade instead of per add) returns the plain loop's bits on 200 000 random
    and edge cases (acc 0 / negative / at a binade edge, ties, tiny and large
    terms), compiled here as plain C++ (the kernels include the same header)."""
    import subprocess
    exe = tmp_path / "exact"
    subprocess.check_call(["g++", "-O2", "-ffp-contract=off", "-std=c++20", "-I",
                           os.path.join(PKG, "csrc"), os.path.join(ROOT, "tests", "exact_harness.cpp"), "-o", str(exe)])
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "0 / 200000 mismatches" in out.stdout


def test_lazy_longterm_bound(tmp_path):
    """The device VADMachine's lazy long-term test (fvad_staged.hip vadm_stream
    via fvad_exact.h lt_bound / lt_decide / lt_estimate, the code the kernel
    compiles) decides exactly as the reference's st_avg > RN(avg * f)
    (VADMachine.zig:150-167, RollingAverage.zig:45-56) on 2 * 10^6 adversarial
    decisions: st_avg at the exact threshold and +-1, +-2 ulps of it, at the
    bound's window edges +-1, +-2 ulps, over value streams spanning 70 binades
    and owed runs up to 4096 pushes.  Every settled decision matches, and the
    estimate stays within a quarter of E.  With E scaled by 10^-3 the same
    harness finds mismatches: it is sharp enough to catch a bound that is too
    tight."""
    import re
    import subprocess
    exe = tmp_path / "ltb"
    subprocess.check_call(["g++", "-O2", "-ffp-contract=off", "-std=c++20", "-I",
                           os.path.join(PKG, "csrc"), os.path.join(ROOT, "tests", "lt_bound_harness.cpp"), "-o",
                           str(exe)])
    out = subprocess.run([str(exe), "2000000"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    m = re.search(r"decisions (\d+) settled (\d+) open (\d+) mismatches (\d+) .* max \|approx-fold\|/E (\S+)", out.stdout)
    assert m, out.stdout
    dec, settled, opened, bad, worst = int(m[1]), int(m[2]), int(m[3]), int(m[4]), float(m[5])
    assert dec >= 2000000 and bad == 0 and settled > 0.3 * dec and opened > 0.3 * dec, out.stdout
    assert worst < 0.5, out.stdout
    sharp = subprocess.run([str(exe), "200000", "1e-3"], capture_output=True, text=True, timeout=120)
    assert sharp.returncode == 1 and "MISMATCH" in sharp.stdout, sharp.stdout
