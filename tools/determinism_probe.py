"""Diagnostic: run the configs[4]-size engine twice from reset and report
which outputs differ (and where).  Usage: python tools/determinism_probe.py [B] [T]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "formula-vad_amd"))
import fvad

B = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
T = int(sys.argv[2]) if len(sys.argv) > 2 else 24
m = fvad.Model(seed=1)
eng = fvad.Engine(m, B, 2, max_ticks=T, want_denoised=True)
eng.load_synthetic(T, base=0)
outs = []
for r in range(3):
    eng.reset()
    eng.run_resident(T)
    eng.sync()
    outs.append(eng.fetch(T, denoised=True))
for r in (1, 2):
    for k in outs[0]:
        a, b = outs[0][k], outs[r][k]
        d = a != b
        if k != "win_flag":
            d &= ~(np.isnan(a) & np.isnan(b))
        if d.any():
            idx = np.argwhere(d)
            print("run0 vs run%d %-9s differs at %d entries; ticks %s streams %s" %
                  (r, k, d.sum(), np.unique(idx[:, 0])[:10], np.unique(idx[:, 1])[:10]))
            i = tuple(idx[0])
            print("   first", i, a[i], b[i])
print("done")
