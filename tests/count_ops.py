"""Instrumented work counts of the bench workload (test infrastructure: runs
the oracle, never imported by the product).

The bench (bench.py) re-runs one resident push of 50 ticks of the synthetic
streams fvad_synth_stream(base + s) per step.  This runs the same input through
the oracle's whole per-stream path (ora_bench_pipeline: rnnoise + FFT B +
VADMachine) for a strided sample of the 2048 streams, 4 pushes each, and
counts per channel-frame what the algorithm actually does where its work is
data dependent:

  fine_lags   pitch_search's fine xcorr lags (|i - 2 best| <= 2 for either of
              the two coarse candidates: 5..10 per frame)
  rd_cands    remove_doubling candidates evaluated (k = 2..15 until T1 <
              minperiod)
  silent      frames under the E < 0.04 gate (no GRU stack, pitch filter or
              gains)

`python tests/count_ops.py` prints the dict committed as
formula-vad_amd/fvad/cost.py MEASURED; tests/test_host_cpu.py recounts it.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "oracle"), os.path.join(ROOT, "formula-vad_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

STREAMS, STRIDE, TICKS, PUSHES, CHANNELS = 256, 8, 50, 4, 2


def count(streams=STREAMS, stride=STRIDE, ticks=TICKS, pushes=PUSHES, channels=CHANNELS, threads=8):
    import numpy as np
    import fvad
    import oracle
    n = ticks * 480
    pcm = np.zeros((streams, channels, n * pushes), np.float32)
    for i in range(streams):
        x, _ = fvad.synth_stream(i * stride, n, channels)
        pcm[i] = np.tile(x, (1, pushes))
    _, c = oracle.bench_pipeline(pcm, chunk=n, n_threads=threads)
    f = c["frames"]
    return {"fine_lags_per_frame": round(c["fine_lags"] / f, 4), "rd_cands_per_frame": round(c["rd_cands"] / f, 4),
            "silent_frac": round(c["silent"] / f, 6), "frames_counted": f}


if __name__ == "__main__":
    print(count())
