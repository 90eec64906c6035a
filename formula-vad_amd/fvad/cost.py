"""Algorithmic cost of one channel-frame (480 samples of one channel through
rnnoise, plus its share of FFT B) — the unit of the bench metric.

Counts follow the loop trip counts of the restated algorithm (SURVEY.md
Appendix A / oracle/ora_rnnoise.c): every f32/f64 add, sub, mul, div and sqrt
is one flop; table lookups, copies, compares and max/min are free.  The
data-dependent trip counts (fine-search lags, remove_doubling candidates, the
silence gate) are the instrumented averages of the oracle on the bench's own
input (MEASURED, from tests/count_ops.py), not upper bounds.  The per-phase
breakdown is reproduced in DESIGN.md §5.
"""

FRAME = 480

# tests/count_ops.py on the bench workload (256 of the 2048 synthetic streams,
# the 20 distinct resident 50-tick pushes = their first 10 s, as bench.py
# cycles through them): per channel-frame averages; tests/test_host_cpu.py
# recounts them
MEASURED = {"fine_lags_per_frame": 9.3352, "rd_cands_per_frame": 6.6061, "silent_frac": 0.004516,
            "frames_counted": 512000}
PTILE_ROWS = 8 + 147 + 37 + 1  # k_plpc -> k_pcorr rows per frame (fvad_staged.h ptile: FIR coefficients + x_lp[0],
#   coarse Syy, fine Syy checkpoints, xx; xf is rebuilt by k_pcorr from the x_lp rows)


def _fft960():
    r4_degenerate = 240 * 16          # 16 adds per m=1 butterfly
    r4_general = 2 * 240 * (3 * 6 + 16)  # 3 complex muls + 16 adds, two stages
    r3 = 320 * 28
    r5 = 192 * 72
    return r4_degenerate + r4_general + r3 + r5  # 42944


def _band_sum():
    # per bin: |.|^2 or re/im product (3), weighted into two bands (2 mul, 2 add, 1 sub)
    return 400 * 8


def _fftb_per_window(nfft=2048, n_bins=61):
    nc = nfft // 2
    stages = 0
    n = nc
    while n > 1:
        n //= 4
        stages += 1
    fft = stages * (nc // 4) * (3 * 6 + 16)
    window = nfft
    post = n_bins * (2 + 2 + 6 + 2 + 2)  # fpnk/f1k/f2k, super-twiddle cmul, halves
    mag = n_bins * 4                     # r^2 + i^2, sqrt, norm
    band = n_bins
    return fft + window + post + mag + band


def gru_flops(nin, nout):
    macs = 3 * nout * (nin + nout)
    extra = nout * nout            # (w*state)*r in the candidate gate
    act = 3 * nout * 10 + nout * 4  # activations + state update
    return 2 * macs + extra + act


def phases(n_channels=2, fft_size=2048, counts=None):
    m = counts or MEASURED
    fine, rd, live = m["fine_lags_per_frame"], m["rd_cands_per_frame"], 1.0 - m["silent_frac"]
    p = {}
    p["prep: s16 scale + HP biquad + rms"] = FRAME * (1 + 1 + 3 + 4 + 2) + 2
    p["analysis window + FFT A + scale"] = 960 + 1920 + _fft960()
    p["band energy Ex"] = _band_sum()
    p["pitch downsample + autocorr + LPC + FIR5"] = 864 * 4 + 5 * 864 * 2 + 60 + 864 * 10
    p["coarse xcorr 147x240 + find_best_pitch"] = 147 * 240 * 2 + 240 * 2 + 147 * 8
    p["fine xcorr <=10x480 + find_best_pitch"] = fine * 480 * 2 + 480 * 2 + 294 * 8
    p["remove_doubling"] = 480 * 4 + 480 * 2 + 384 * 4 + rd * 480 * 4 + 3 * 480 * 2 + rd * 12
    p["pitch window + FFT + Ep + Exp"] = 960 + 1920 + _fft960() + 2 * _band_sum() + 22 * 5
    p["features (log10, DCTs, cepstra, spectral variability)"] = 22 * 3 + 28 * 44 + 18 * 3 + 8 * 8 * 22 * 3 + 16
    # skipped on frames under the silence gate (denoise.c: if (!silence))
    p["GRU stack"] = live * ((2 * 42 * 24 + 24 * 10) + gru_flops(24, 24) + 2 * 24 + gru_flops(90, 48) +
                             gru_flops(114, 96) + (2 * 96 * 22 + 22 * 12))
    p["pitch filter + gains"] = live * (22 * 20 + 481 * 7 + _band_sum() + 22 * 6 + 481 * (2 * 3 + 4))
    p["synthesis (scale, FFT A, window, OLA, 1/32767)"] = 1920 + _fft960() + 960 + 960 + 480 + 480
    p["re-block + FFT B share"] = _fftb_per_window(fft_size) * FRAME / fft_size + 4
    p["VADMachine share"] = _vadm_per_window() * FRAME / fft_size / n_channels
    return p


def _vadm_per_window(n_lt=4218, n_st=4, n_r=11):
    """VADMachine.run per window and stream: the three RollingAverage means are
    recomputed over their whole buffers (mul + add per entry, f64); the
    long-term one only outside speech (counted as always, the upper bound)."""
    return 2 * (n_lt + n_st + n_r) + 24


def flops_per_channel_frame(n_channels=2, fft_size=2048):
    return sum(phases(n_channels, fft_size).values())


def path_bytes_per_channel_frame(n_channels=2, state_bytes=12236):
    """SURVEY.md §8(d) B_alg, the real-time tick model: input 1920 B + vad 4 B
    + band ~1 B + the rnnoise state read and written once per stream-tick
    (shared by the C channels) + the FFT-B carry of the denoised frame written
    and read (3840 B)."""
    return 1920 + 4 + 1 + 2.0 * state_bytes / n_channels + 3840


def frame_kernel_bytes(n_streams, n_channels, n_ticks, n_bands=1, state_words=2816, live_state_words=2788,
                       fft_size=2048):
    """Algorithmic HBM bytes of one k_frame launch (T ticks of B streams)."""
    B, C, T = n_streams, n_channels, n_ticks
    frames = T * B * C
    xbuf = frames * FRAME * 4
    ratio = T * B * 4
    state = 2 * B * live_state_words * 4
    ring_w = frames * FRAME * 4
    ring_r = frames * FRAME * 4  # every denoised sample is read once by FFT B
    outs = T * B * (4 * 4 + C * n_bands * 4)
    return xbuf + ratio + state + ring_w + ring_r + outs


def prep_kernel_bytes(n_streams, n_channels, n_ticks):
    frames = n_streams * n_channels * n_ticks
    return frames * FRAME * 4 * 2 + n_streams * n_ticks * 4 + n_streams * 16


def staged_kernels(n_channels=2, fft_size=2048):
    """Per channel-frame algorithmic flops and HBM bytes of each staged kernel
    (fvad_staged.hip).  Flops re-partition phases() (the sum is unchanged);
    bytes are the kernel's compulsory reads + writes of its inputs/outputs in
    the staged layout.  k_pcorr's speculative work (the
    final 3-lag xcorr for every candidate instead of the selected one) is
    counted once, as the reference computes it."""
    p = phases(n_channels, fft_size)
    rd = MEASURED["rd_cands_per_frame"]
    C = n_channels
    feat = p["features (log10, DCTs, cepstra, spectral variability)"]
    dct_ly = 22 * 44 + 22 * 2
    dct_exp = 6 * 44 + 6 * 2
    spec = 481 * 8  # one complex spectrum
    pitch = (p["pitch downsample + autocorr + LPC + FIR5"] + p["coarse xcorr 147x240 + find_best_pitch"] +
             p["fine xcorr <=10x480 + find_best_pitch"] + p["remove_doubling"] - rd * 12)
    # k_plpc: x_lp, autocorr, LPC, FIR and the serial energy recurrences of
    # both find_best_pitch scans (Syy init + updates) and xx; k_pcorr the rest,
    # remove_doubling's yy_lookup recurrence included (r2)
    # x_lp itself (864 * 4 per frame in the reference) is computed once per
    # push position: k_fftAw writes each frame's 240 new values into the x_lp
    # rows (k_prep3 the history's), so the term is charged to k_fftAw
    xlp = 864 * 4
    plpc = (p["pitch downsample + autocorr + LPC + FIR5"] - xlp + 240 * 2 + 147 * 4 + 480 * 2 + 294 * 4 +
            480 * 2)
    k = {
        "k_prep3": (p["prep: s16 scale + HP biquad + rms"], 480 * 4 * 2 + 4.0 / C),
        "k_fftAw": (p["analysis window + FFT A + scale"] + p["band energy Ex"] + 22 * 3 + dct_ly + xlp,
                   960 * 4 + spec + 22 * 4 * 2 + 4 + 240 * 4),
        # k_plpc: the frame's x_lp window (+ 2 pitch-buffer samples for x_lp[0])
        # in; the FIR coefficients, the coarse Syy sequence, the fine Syy
        # checkpoints and xx out (r3: xf and yy_lookup no longer go through HBM).
        # k_pcorr: the x_lp window + that tile row in (2 fine checkpoints), the
        # pitch record out
        "k_plpc": (plpc, (864 + 2) * 4 + PTILE_ROWS * 4),
        "k_pcorr": (pitch - xlp - plpc - rd * 4, (864 + 6 + 147 + 2 + 1) * 4 + 80 * 4),
        "k_select": (rd * 4 + rd * 12, 80 * 4 + 4),
        "k_pspecw": (p["pitch window + FFT + Ep + Exp"] + dct_exp, 960 * 4 + 2 * spec + 22 * 4 * 3 + 8 * 4 + 4),
        # k_rnn3: cepstral memory, spectral variability, GRU stack, gain
        # smoothing; reads DCT(Ly), features 34..40, silence; writes g, smoothed g, vad
        "k_rnn3": (feat - 22 * 3 - dct_ly - dct_exp + p["GRU stack"],
                  (22 + 8 + 1) * 4 + (22 + 22 + 1) * 4),
        # k_synthw: pitch filter (X + r P, band energies, norm), gains, synthesis;
        # reads X, P, Exp, g, Ex, Ep, smoothed g, silence; writes the windowed frame
        "k_synthw": (p["pitch filter + gains"] + p["synthesis (scale, FFT A, window, OLA, 1/32767)"] - 960,
                    2 * spec + 5 * 22 * 4 + 4 + 960 * 4),
        "k_ola": (960, 960 * 4 + 480 * 4 + 4.0 / C),
        "k_winmeta": (0.0, 4 * 4.0 / C),
        "k_fftbw": (p["re-block + FFT B share"], 480 * 4 + 4),
        # fft_size 512: the workgroup-per-window kernel, same work
        "k_fftb": (p["re-block + FFT B share"], 480 * 4 + 4),
        "k_vadm_hbm": (p["VADMachine share"], (4218 + 4 + 11 + 2) * 4 * FRAME / fft_size / C + 16),
    }
    # k_olafb (fft_size 2048, <= 4 channels): k_ola + k_winmeta + k_fftbw in one
    # kernel; the ys rows in, per-tick outputs out, the re-block window stays
    # in LDS (only the partial window crosses pushes through the ring:
    # <= 2047 samples each way per channel and push, ~2 x 8 KB / 50 ticks)
    k["k_olafb"] = (960 + p["re-block + FFT B share"], 960 * 4 + 4 * 4.0 / C + 2 * 8192.0 / 50)
    k["k_vadm_par"] = k["k_vadm_hbm"]  # the same machine, window-parallel (the push flushed at a sync point)
    k["k_gru16"] = k["k_rnn3"]  # FVAD_MODE_FP16: the same recurrence, gate sums on MFMA
    # FVAD_MODE_FP16_FUSED: k_pspecw's work and k_gru16's in one kernel; features
    # 34..40 pass in LDS, so the f34 row (8 floats) is neither written nor read
    k["k_fused16"] = (k["k_pspecw"][0] + k["k_rnn3"][0], k["k_pspecw"][1] + k["k_rnn3"][1] - 2 * 8 * 4)
    return {n: {"flops": f, "bytes": b} for n, (f, b) in k.items()}


if __name__ == "__main__":
    for k, v in phases().items():
        print("%-58s %9d" % (k, v))
    print("%-58s %9d" % ("TOTAL flops / channel-frame", flops_per_channel_frame()))
