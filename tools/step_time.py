"""Diagnostic: wall time per push of the bench workload (2048 stereo streams,
50 ticks, device VADMachines), without the bench's roofline bookkeeping.
Usage: [FVAD_NO_EVENTS=1] python3 tools/step_time.py [steps]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "formula-vad_amd"))
import fvad

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
B, C, T = 2048, 2, 50
eng = fvad.Engine(fvad.Model(seed=1), B, C, max_ticks=T)
eng.attach_vadm()
eng.load_synthetic(T)
for _ in range(3):
    eng.run_resident(T)
eng.sync()
t0 = time.perf_counter()
for _ in range(steps):
    eng.run_resident(T)
eng.sync()
dt = (time.perf_counter() - t0) / steps
print("events=%s ms/push %.3f  frames/s %.1fM" % (os.environ.get("FVAD_NO_EVENTS", "0") != "1", dt * 1e3,
                                                   B * C * T / dt / 1e6))
