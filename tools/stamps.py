"""Diagnostic: per-phase cycle shares of k_frame (fused mode) or k_rnn
(staged mode) from the FVAD_STAMPS build.
Usage: FVAD_LIB=formula-vad_amd/lib/libfvad_stamps.so python tools/stamps.py [streams] [ticks] [fused|staged]
Shares only — the stamp build's fences distort absolute time."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "formula-vad_amd"))
import fvad

NAMES = ["load state", "pitch shift", "analysis window+scatter", "FFT A (X) + copy", "Ex + downsample",
         "autocorr", "LPC", "FIR5", "coarse xcorr + Syy seqs", "coarse scan", "fine xcorr", "fine scan",
         "remove_doubling products", "rd selection", "rd final xcorr", "P window+FFT+Ep/Exp",
         "Exp norm/log10/DCT/Ly", "features", "dense + vad GRU", "noise GRU", "denoise GRU + out",
         "pitch filter + gains", "synthesis", "tick end + FFT B"]
B = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
T = int(sys.argv[2]) if len(sys.argv) > 2 else 20
MODE = sys.argv[3] if len(sys.argv) > 3 else "fused"
if MODE == "staged":  # k_rnn3 (the only staged recurrence kernel since r2)
    NAMES = ["P1 z|r gates + spectral variability(t) + gains(t-5)",
             "P2 candidates, dense(t), outputs, features(t+1)",
             "  P1 role: denoise z|r", "  P1 role: noise z|r", "  P1 role: vad z|r", "  P1 role: spectral var",
             "  P1 role: gains", "", "  P2 role: denoise h", "  P2 role: noise h", "  P2 role: vad h",
             "  P2 role: dense", "  P2 role: denoise_output", "  P2 role: vad_output", "  P2 role: features"]
    ROLES = True
if MODE in ("fp16", "fp16_fused"):  # k_gru16 / k_fused16 supersteps (fvad_gru16.hip), stamps[48..49]
    GRU = ["A  z|r gates vad(u-1) noise(u-2) denoise(u-3), dense(u), outputs, features(u+1)",
           "B  candidates vad(u-1) noise(u-2) denoise(u-3), gains(u-4), spectral var(u+1)"
           + (", pitch spectrum(u+2)" if MODE == "fp16_fused" else "")]
L = fvad.lib()
L.fvad_engine_stamps.restype = C.c_int
L.fvad_engine_stamps.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong), C.c_int]
m = fvad.Model(seed=1)
e = fvad.Engine(m, B, 2, max_ticks=T, mode=MODE)
e.load_synthetic(T)
e.run_resident(T)
e.sync()
assert L.fvad_engine_stamps(e.h, None, 0) == 0  # allocate + zero
e.run_resident(T)
e.sync()
buf = (C.c_ulonglong * 128)()
assert L.fvad_engine_stamps(e.h, buf, 128) == 0
if MODE in ("fp16", "fp16_fused"):
    frames = (B // 8) * 2 * T  # one workgroup per 8 streams (kSpw), stamps from thread 0
    gt = sum(buf[48:48 + len(GRU)])
    print("k_gru16" if MODE == "fp16" else "k_fused16", end="")
    print(": stamped cycles per frame step per WG: %.0f" % (gt / frames))
    for i, n in enumerate(GRU):
        print("%2d %-44s %6.2f%%  %8.0f cyc/frame" % (i, n, 100.0 * buf[48 + i] / max(1, gt), buf[48 + i] / frames))
    print("per-wave busy cycles per frame step (phase A | phase B):")
    for w in range(8):
        print("  w%d %8.0f | %8.0f" % (w, buf[w] / frames, buf[8 + w] / frames))
    if MODE == "fp16_fused":
        print("pitch-spectrum waves (phase A: transform of u+2 | phase B: its features):")
        for w in range(8):
            print("  w%d %8.0f | %8.0f" % (8 + w, buf[16 + w] / frames, buf[24 + w] / frames))
    sys.exit(0)
tot = sum(buf[:24]) if MODE == "fused" else (sum(buf[:2]) if len(NAMES) > 12 else sum(buf[:12]))
frames = B * 2 * T
if MODE == "staged":
    frames = (B // 8) * 2 * T  # k_rnn: one workgroup per 8 streams, stamps = frame steps of thread 0
print("total stamped cycles per frame step per WG: %.0f" % (tot / frames))
for i, n in enumerate(NAMES[:24]):
    if not n:
        continue
    print("%2d %-28s %6.2f%%  %8.0f cyc/frame" % (i, n, 100.0 * buf[i] / tot, buf[i] / frames))
if MODE == "fused":
    print("   %-28s %6.2f%%" % ("store state", 100.0 * buf[23] / tot if len(buf) > 23 else 0))
if MODE == "staged":
    print("k_rnn3 per-wave busy cycles per frame step (P1 | P2):")
    for w in range(16):
        print("  w%-2d %8.0f | %8.0f" % (w, buf[64 + w] / frames, buf[80 + w] / frames))

if MODE == "staged":
    PIT = ["Q0 xf + coarse Syy -> LDS", "Q1 coarse xcorr", "Q2 coarse scan (survivors)", "Q3 fine xcorr",
           "Q4 fine scan", "Q5 remove_doubling products"]
    groups = B * 2 * T / 8.0
    pt = sum(buf[32:38])
    print("k_pcorr: stamped cycles per 8-frame group per WG: %.0f" % (pt / max(1, groups)))
    for i, n in enumerate(PIT):
        print("%2d %-32s %6.2f%%  %8.0f cyc/group" % (i, n, 100.0 * buf[32 + i] / max(1, pt), buf[32 + i] / groups))
    print("   alone: coarse scan %8.0f, yy walk (wave 2, Q2..Q4) %8.0f cyc/group" % (buf[38] / groups, buf[39] / groups))

if MODE == "staged":
    SYN = ["setup + X load + pitch gain r", "pitch filter + band terms", "band chains, norm, gains",
           "Hermitian staging", "FFT + synthesis window out"]
    groups = B * 2 * T / 4.0
    tt = sum(buf[40:45])
    print("k_synth: stamped cycles per 4-frame group per WG: %.0f" % (tt / max(1, groups)))
    for i, n in enumerate(SYN):
        print("%2d %-32s %6.2f%%  %8.0f cyc/group" % (i, n, 100.0 * buf[40 + i] / max(1, tt), buf[40 + i] / groups))
