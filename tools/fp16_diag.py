"""GPU diagnostic (not collected by pytest): fp16 engine mode vs the oracle --
error statistics that set the tolerances of tests/test_gpu_fp16.py."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import conftest  # noqa: F401 (sys.path)
import numpy as np
import fvad
import oracle
import parity_util as pu

oracle.build()
m, om = fvad.Model(seed=1), oracle.Model(seed=1)
ids = [0, 1, 19, 42, 7]
streams = [fvad.synth_stream(i, 48000 * 20, 2)[0] for i in ids]
ref = pu.oracle_run(oracle, om, streams)
for mode in ("staged", "fp16"):
    eng = fvad.Engine(m, len(ids), 2, max_ticks=50, want_denoised=True, mode=mode)
    got = pu.engine_run(fvad, eng, streams, 50)
    for s, (r, g) in enumerate(zip(ref, got)):
        fr = r["frames"]
        dv = np.abs(fr["vad"] - g["vad"])
        dr, dg = r["denoised"], g["denoised"]
        rel = np.sqrt(np.mean((dr - dg) ** 2)) / np.sqrt(np.mean(dr ** 2))
        wi = r["windows"]
        b = np.abs(wi["band"][:, :2] - g["band"][:, :, 0]).max() / np.abs(wi["band"][:, :2]).max()
        print("%-6s stream %3d: vad max|d| %.3e mean %.3e  den relRMS %.3e  band rel %.3e  ratio eq %s" % (
            mode, ids[s], dv.max(), dv.mean(), rel, b, np.array_equal(fr["ratio"], g["ratio"])), flush=True)
