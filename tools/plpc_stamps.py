"""Diagnostic: k_plpc per-pass cycle totals from the FVAD_STAMPS build
(stamps[56..59], lane 0 of every workgroup's wave 0).
Usage: FVAD_LIB=formula-vad_amd/lib/libfvad_stamps.so python tools/plpc_stamps.py [streams] [ticks]"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "formula-vad_amd"))
import fvad

B = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
T = int(sys.argv[2]) if len(sys.argv) > 2 else 50
L = fvad.lib()
L.fvad_engine_stamps.restype = C.c_int
L.fvad_engine_stamps.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong), C.c_int]
e = fvad.Engine(fvad.Model(seed=1), B, 2, max_ticks=T, mode="staged")
e.load_synthetic(T)
e.run_resident(T)
e.sync()
assert L.fvad_engine_stamps(e.h, None, 0) == 0
e.run_resident(T)
e.sync()
buf = (C.c_ulonglong * 64)()
assert L.fvad_engine_stamps(e.h, buf, 64) == 0
tiles = (B + 63) // 64 * T * 2
names = ["pass 1 (autocorr)", "pass 2 (FIR, Syy)", "pass 3 (yy)", "setup"]
tot = sum(buf[56:60])
for i, n in enumerate(names):
    print("k_plpc %-20s %6.1f%%  %8.0f cyc/tile" % (n, 100.0 * buf[56 + i] / max(1, tot), buf[56 + i] * 4.0 / tiles))
