"""bench.py's host-fed legs (host_rate) on a simulated engine, CPU only: the
fill-inclusive figure (20 pushes from an empty pipeline) and the steady-state
one (push periods between collects with FVAD_MAX_IN_FLIGHT pushes kept in
flight) must come out as the pipeline model says.  The fake engine completes
push k at max(its submit time + latency, completion of push k-1 + period), so
the steady state is the period and the fill-inclusive rate pays the first
push's latency once."""
import os
import sys
import time

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PERIOD, LATENCY = 0.012, 0.030  # s (LATENCY < 3 PERIOD: three in flight keep the period)


class FakeEngine:
    def __init__(self, T, B, C):
        self.slot = np.zeros((3, T, B, C, 480), np.float32)
        self.slot16 = np.zeros((3, T, B, C, 480), np.int16)
        self.k = 0
        self.done = []  # completion times of submitted, uncollected pushes
        self.last = 0.0

    def input_slot(self):
        return self.slot[self.k % 3]

    def input_slot_i16(self):
        return self.slot16[self.k % 3]

    def _submit(self):
        t = time.perf_counter()
        self.last = max(t + LATENCY, self.last + PERIOD)
        self.done.append(self.last)
        self.k += 1

    def submit(self, pcm):
        self._submit()

    def submit_i16(self, pcm):
        self._submit()

    def collect(self, want=True):
        t = self.done.pop(0)
        while time.perf_counter() < t:
            time.sleep(0.0005)


class FakeGroup:
    def __init__(self, T, B, C):
        self.engines = [FakeEngine(T, B, C)]
        self.first, self.sizes, self.B = [0], [B], B

    def sync(self):
        for e in self.engines:
            while e.done:
                e.collect()


def test_host_rate_steady_and_fill():
    sys.path.insert(0, ROOT)
    import bench

    class A:
        channels, ticks, steps, resident_pushes = 2, 2, 20, 20
    grp = FakeGroup(A.ticks, 4, A.channels)
    res = bench.host_rate(grp, A, 0, None, None, 0)
    steady = res["steady_ms_per_step"]
    for kind in ("pinned", "pageable", "pinned_i16"):
        assert steady[kind] == pytest.approx(1000 * PERIOD, rel=0.15), (kind, steady)
    # the fill-inclusive figures pay the first push's latency (and the drain) once
    fill = 1000 * (LATENCY + (A.steps - 1) * PERIOD) / A.steps
    for key in ("ms_per_step", "pageable_ms_per_step", "i16_ms_per_step"):
        assert res[key] == pytest.approx(fill, rel=0.15), (key, res[key], fill)
        assert res[key] > steady["pinned"]
