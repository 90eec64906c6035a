"""Device VADMachine timing in the bench schedule (2048 streams, 50-tick pushes,
the resident 10 s cycle), twice: as the bench runs it (streams in their first
seconds: the long-term RollingAverage still holds initial entries, which
k_vadm's recompute adds per binade, fvad_exact.h) and with every long-term
entry counted as pushed (FVAD_DEBUG_VADM_LT_FULL: a stream past its first
180 s, the recompute walks ~4 200 stored entries per window).  Timing only:
with the hook the values are not the reference's.
Usage (GPU box): python3 tools/vadm_steady.py"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "formula-vad_amd"))
import fvad

B, C, T, P = 2048, 2, 50, 20
m = fvad.Model(seed=1)
out = {}
PAR = int(os.environ.get("VADM_PAR_BOTH", "0"))
RUNS = (("bench_first_seconds", 0, 0), ("long_term_full", 1, 0), ("bench_first_seconds_par", 0, 1),
        ("long_term_full_par", 1, 1))[:4 if PAR else 2]
if os.environ.get("VADM_ONLY_FULL"):
    RUNS = [r for r in RUNS if r[1]]
for name, full, par in RUNS:
    e = fvad.Engine(m, B, C, max_ticks=T)
    e.attach_vadm()
    if full:
        e.set_debug(fvad.DEBUG_VADM_LT_FULL, 1)
    if par:  # every push's machine on k_vadm_par (FVAD_DEBUG_VADM_ALWAYS_PAR)
        e.set_debug(fvad.DEBUG_VADM_ALWAYS_PAR, 1)
    e.load_synthetic(T, base=0, pushes=P)
    for _ in range(5):
        e.run_resident(T)
    e.sync()
    e.clear_times()
    t0 = time.perf_counter()
    for _ in range(20):
        e.run_resident(T)
    e.sync()
    wall = (time.perf_counter() - t0) / 20 * 1000
    kt = e.kernel_times()
    out[name] = {"ms_per_push": round(wall, 4),
                 "kernels_ms": {k: round(v, 4) for k, v in kt["kernels"].items()}}
    del e
print(json.dumps(out))
