"""Ad-hoc GPU diagnostic (not collected by pytest): engine vs oracle on a few streams."""
import sys, os, time
sys.path.insert(0, os.path.dirname(__file__))
import conftest  # noqa: F401 (sys.path)
import numpy as np
import fvad, oracle
import parity_util as pu

oracle.build()
secs = float(sys.argv[1]) if len(sys.argv) > 1 else 6
ids = [0, 1, 19]
m = fvad.Model(seed=1)
om = oracle.Model(seed=1)
streams, labels = pu.make_streams(fvad, ids, secs)
t = time.time()
ref = pu.oracle_run(oracle, om, streams)
print("oracle %.1fs" % (time.time() - t), flush=True)
eng = fvad.Engine(m, len(ids), 2, max_ticks=50, want_denoised=True)
t = time.time()
got = pu.engine_run(fvad, eng, streams, 50)
print("engine %.1fs" % (time.time() - t), flush=True)
for s in range(len(ids)):
    r, g = ref[s], got[s]
    fr = r["frames"]
    print("stream", ids[s], "frames", len(fr), len(g["vad"]))
    print("  vad  max|d|", np.abs(fr["vad"] - g["vad"]).max(), "first mismatch", pu.first_mismatch(fr["vad"], g["vad"]))
    print("  ratio max|d|", np.abs(fr["ratio"] - g["ratio"]).max(), pu.first_mismatch(fr["ratio"], g["ratio"]))
    dr, dg = r["denoised"], g["denoised"]
    print("  den  max|d|", np.abs(dr - dg).max(), "rel", np.abs(dr - dg).max() / max(1e-30, np.abs(dr).max()),
          "first", pu.first_mismatch(dr, dg))
    wi = r["windows"]
    print("  windows", len(wi), int(g["win_flag"].sum()))
    n = min(len(wi), len(g["band"]))
    if n:
        print("  band max|d|", np.abs(wi["band"][:n, :2] - g["band"][:n, :, 0]).max(),
              "ratio", np.abs(wi["ratio"][:n] - g["win_ratio"][:n]).max(),
              "vad", np.abs(wi["vad"][:n] - g["win_vad"][:n]).max())
