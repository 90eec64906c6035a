#!/usr/bin/env python3
"""BASELINE configs[1]: one 48 kHz stereo stream on one MI355X.  Times the
staged engine (device VADMachine attached) on pushes of 1, 10 and 50 ticks
(10 ms, 100 ms, 0.5 s of audio) from host memory (fvad_engine_push: H2D,
kernels, outputs back, synchronous), and reports ms per push and the
real-time factor (audio seconds per wall second).  One JSON line."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "formula-vad_amd"))


def main():
    import fvad
    model = fvad.Model(seed=1)
    res = {}
    for T in (1, 10, 50):
        eng = fvad.Engine(model, 1, 2, max_ticks=T)
        eng.attach_vadm()
        x = fvad.synth_stream(0, 48000 * 20, 2)[0]
        n = x.shape[1] // (480 * T)
        pushes = [np.ascontiguousarray(x[:, k * T * 480:(k + 1) * T * 480].reshape(2, T, 480).transpose(1, 0, 2)
                                       [:, None]) for k in range(n)]
        for p in pushes[:5]:
            eng.push(p)
        eng.sync()
        reps = min(n - 5, 200)
        t0 = time.perf_counter()
        for p in pushes[5:5 + reps]:
            eng.push(p)
        eng.sync()
        dt = (time.perf_counter() - t0) / reps
        res["ticks_%d" % T] = {"ms_per_push": round(1000 * dt, 3), "audio_ms": 10 * T,
                               "realtime_factor": round(0.01 * T / dt, 1)}
        del eng
    print(json.dumps({"config": "BASELINE configs[1]: 1 stereo 48 kHz stream, staged engine, device VADMachine, "
                                "synchronous fvad_engine_push from host memory", "results": res}))


if __name__ == "__main__":
    main()
