"""Instrumented work counts of the bench workload (test infrastructure: runs
the oracle, never imported by the product).

The bench (bench.py) cycles through 20 resident pushes of 50 ticks: the first
10 s of the synthetic streams fvad_synth_stream(base + s) (generated at that
length); with --warmup 5 --steps 20 the timed pushes are exactly one cycle.
This runs the same input through the oracle's whole per-stream path
(ora_bench_pipeline: rnnoise + FFT B + VADMachine) for a strided sample of the
2048 streams, in 50-tick pushes, and counts per channel-frame what the
algorithm actually does where its work is data dependent:

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

STREAMS, STRIDE, TICKS, PUSHES, CHANNELS = 256, 8, 50, 20, 2


def count(streams=STREAMS, stride=STRIDE, ticks=TICKS, pushes=PUSHES, channels=CHANNELS, threads=8):
    import numpy as np
    import fvad
    import oracle
    n = ticks * 480
    pcm = np.zeros((streams, channels, n * pushes), np.float32)
    for i in range(streams):
        # stride-8 ids shifted by i % 8, so the sample includes the every-20th
        # stream with digital silence (ids = 19 mod 20 are odd)
        pcm[i], _ = fvad.synth_stream(i * stride + i % stride, n * pushes, channels)
    _, c = oracle.bench_pipeline(pcm, chunk=n, n_threads=threads)
    f = c["frames"]
    return {"fine_lags_per_frame": round(c["fine_lags"] / f, 4), "rd_cands_per_frame": round(c["rd_cands"] / f, 4),
            "silent_frac": round(c["silent"] / f, 6), "frames_counted": f}


if __name__ == "__main__":
    print(count())
