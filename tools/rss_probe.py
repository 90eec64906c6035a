"""Diagnostic: this process's resident set (VmRSS, MB) after each step of the
bench's host-side life (bench.py host_memory), to attribute what is not the
pinned slots.  Usage: python3 tools/rss_probe.py  (needs a GPU)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "formula-vad_amd"))
import fvad  # noqa: E402


KEYS = ("VmRSS", "RssAnon", "RssFile", "RssShmem")


def rss():
    with open("/proc/self/status") as f:
        kb = {ln.split(":")[0]: int(ln.split()[1]) for ln in f if ln.startswith(tuple(k + ":" for k in KEYS))}
    return [kb.get(k, 0) / 1024.0 for k in KEYS]


last = [rss()]
print("%-34s " % "stage" + " ".join("%18s" % k for k in KEYS))


def stage(name):
    r = rss()
    print("%-34s " % name + " ".join("%8.1f (%+8.1f)" % (v, v - w) for v, w in zip(r, last[0])), flush=True)
    last[0] = r


stage("start (numpy + fvad imported)")
m = fvad.Model(seed=1)
stage("model")
tiny = fvad.Engine(m, 1, 2, max_ticks=1)
stage("1-stream engine (HIP runtime up)")
del tiny
stage("1-stream engine destroyed")
B, Ch, T = 2048, 2, 50
e = fvad.Engine(m, B, Ch, max_ticks=T)
stage("2048-stream engine")
e.attach_vadm()
stage("attach_vadm")
e.load_synthetic(T, base=0, pushes=20)
stage("load_synthetic 20 pushes")
for _ in range(3):
    e.run_resident(T)
e.sync()
stage("3 resident pushes")
sl = e.input_slot()[:T]
stage("input_slot 0 (pinned)")
fvad.synth_ticks(0, B, Ch, 20 * T, 0, T, out=sl)
stage("synth into slot 0")
e.submit(sl)
e.collect(want=False)
e.sync()
stage("submit/collect slot 0")
pages = np.array(sl)
stage("pageable copy of one push")
for _ in range(3):
    e.submit(pages)
    e.collect(want=True)
e.sync()
stage("3 pageable submits")
del pages
stage("pageable array freed")
s16 = e.input_slot_i16()[:T]
for t in range(T):
    s16[t] = np.clip(np.round(sl[t] * np.float32(32768.0)), -32768, 32767)
e.submit_i16(s16)
e.collect(want=False)
e.sync()
stage("i16 slot filled + submitted")
del e
stage("engine destroyed")
