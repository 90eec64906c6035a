"""Diagnostic: several engines in one process sharing one GPU, pushing
concurrently (each its own main stream), against one engine over all the
streams.  Env: PROBE_CFG="n_eng:streams_each,..." (default "1:2048,2:1024,2:2048"),
PROBE_SHARE (fvad_engine_share_streams bits for engines 1.. with engine 0:
1 k_prep3's stream, 2 the VADMachine's; default 3), run under different
GPU_MAX_HW_QUEUES to see whether the engines' streams share hardware
queues.  Prints aggregate channel-frames/s per configuration."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "formula-vad_amd"))
import fvad  # noqa: E402

m = fvad.Model(seed=1)
T, P, STEPS = 50, 20, 20
for cfg in os.environ.get("PROBE_CFG", "1:2048,2:1024,2:2048").split(","):
    n_eng, B = (int(x) for x in cfg.split(":"))
    share = int(os.environ.get("PROBE_SHARE", "3"))
    grp = fvad.EngineGroup(m, n_eng * B, 2, groups=n_eng, vadm=True, max_ticks=T)
    engs = grp.engines
    for i, e in enumerate(engs):
        e.load_synthetic(T, base=i * B, pushes=P)
    for _ in range(5):
        for e in engs:
            e.run_resident(T)
    for e in engs:
        e.sync()
    t0 = time.perf_counter()
    for _ in range(STEPS):
        for e in engs:
            e.run_resident(T)
    for e in engs:
        e.sync()
    dt = time.perf_counter() - t0
    print("hwq=%s share=%d %d x %d streams: %.2f M frames/s, %.3f ms per step of all engines" % (
        os.environ.get("GPU_MAX_HW_QUEUES", "-"), share, n_eng, B, n_eng * B * 2 * T * STEPS / dt / 1e6, dt / STEPS * 1e3),
        flush=True)
    del engs, grp
