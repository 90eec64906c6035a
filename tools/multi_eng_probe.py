import sys, time, json
sys.path.insert(0, "formula-vad_amd")
import fvad
m = fvad.Model(seed=1)
T = 50
for n_eng in (1, 2, 4):
    B = 2048 // n_eng
    engs = [fvad.Engine(m, B, 2, max_ticks=T) for _ in range(n_eng)]
    for i, e in enumerate(engs):
        e.load_synthetic(T, base=i * B)
    for _ in range(2):
        for e in engs: e.run_resident(T)
    for e in engs: e.sync()
    t0 = time.perf_counter()
    steps = 10
    for _ in range(steps):
        for e in engs: e.run_resident(T)
    for e in engs: e.sync()
    dt = time.perf_counter() - t0
    print(n_eng, "engines:", round(2048 * 2 * T * steps / dt / 1e6, 2), "M frames/s", round(dt / steps * 1000, 2), "ms/step")
    del engs
