#!/usr/bin/env python3
"""The bench's host-fed leg alone (fvad_engine_submit_i16 / collect, three
pushes in flight, 2048 stereo streams x 50 ticks, device VADMachine), for a
rocprofv3 kernel + memory-copy trace of the ingest timeline:
  rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d DIR -- python3 tools/host_trace.py [--float]
then  python3 tools/host_trace.py --report DIR"""
import glob
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "formula-vad_amd"))


def run(float_in, pushes=16, B=2048, Ch=2, T=50):
    import numpy as np
    import fvad
    eng = fvad.Engine(fvad.Model(seed=1), B, Ch, max_ticks=T)
    eng.attach_vadm()
    src = fvad.synth_ticks(0, B, Ch, 20 * T, 0, 2 * T)
    halves = (src[:T], src[T:])
    q16 = [np.clip(np.round(h * 32768.0), -32768, 32767).astype(np.int16) for h in halves]
    for k in range(3):
        if float_in:
            sl = eng.input_slot()
            sl[:T] = halves[k & 1]
            eng.submit(sl[:T])
        else:
            sl = eng.input_slot_i16()
            sl[:T] = q16[k & 1]
            eng.submit_i16(sl[:T])
    for _ in range(3):
        eng.collect(want=False)
    eng.sync()
    t0 = time.perf_counter()
    inflight = 0
    for k in range(pushes):
        if inflight == 3:
            eng.collect(want=True)
            inflight -= 1
        if float_in:
            eng.submit(eng.input_slot()[:T])
        else:
            eng.submit_i16(eng.input_slot_i16()[:T])
        inflight += 1
    while inflight:
        eng.collect(want=True)
        inflight -= 1
    eng.sync()
    print("%.3f ms per push" % (1000 * (time.perf_counter() - t0) / pushes))


def report(d):
    import csv
    ev = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].split("::")[-1]))
    for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            n = int(r.get("Bytes", r.get("Size", 0)) or 0)
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "%s %.0fMB" % (r["Direction"], n / 1e6)))
    ev.sort()
    t0 = ev[0][0]
    big = [e for e in ev if "MB" not in e[2] or float(e[2].split()[-1][:-2]) > 1]
    for s, e, n in big[-90:]:
        print("%9.3f %9.3f %7.3f  %s" % ((s - t0) / 1e6, (e - t0) / 1e6, (e - s) / 1e6, n))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--report":
        report(sys.argv[2])
    else:
        run("--float" in sys.argv)
