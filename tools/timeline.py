#!/usr/bin/env python3
"""Per-push timeline of the main stream from a rocprofv3 --kernel-trace
database (tools/profile.sh writes gpurun_out/prof_<tag>/trace/*.db):
each kernel's start offset, duration and the gap before it, averaged over
the timed pushes; k_prep3 and k_vadm_hbm (side streams) are shown as
overlap windows.
Usage: python3 tools/timeline.py gpurun_out/prof_<tag>/trace"""
import glob
import os
import sqlite3
import sys
from collections import defaultdict

SIDE = {"k_prep3", "k_vadm_hbm"}


def short(name):
    return name.split("(")[0].replace("void ", "").replace("fvad::", "").split("<")[0]


def main():
    d = sys.argv[1]
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
        c = sqlite3.connect(f)
        rows += [(short(n), s, e) for n, s, e in c.execute("select name, start, end from kernels order by start")]
    rows.sort(key=lambda r: r[1])
    # a push starts at k_fftAw
    pushes, cur = [], None
    for r in rows:
        if r[0] == "k_fftAw":
            cur = [r[1], []]
            pushes.append(cur)
        if cur is not None:
            cur[1].append(r)
    pushes = pushes[1:-1] if len(pushes) > 3 else pushes  # drop the edges
    acc = defaultdict(lambda: [0.0, 0.0, 0.0, 0])
    order = []
    total = 0.0
    for t0, ks in pushes:
        prev_end = t0
        main = [k for k in ks if k[0] not in SIDE]
        for name, s, e in main:
            a = acc[name]
            if name not in order:
                order.append(name)
            a[0] += (s - t0) / 1e6
            a[1] += (e - s) / 1e6
            a[2] += max(0, s - prev_end) / 1e6
            a[3] += 1
            prev_end = max(prev_end, e)
        total += (prev_end - t0) / 1e6
        for name, s, e in ks:
            if name in SIDE:
                a = acc[name]
                if name not in order:
                    order.append(name)
                a[0] += (s - t0) / 1e6
                a[1] += (e - s) / 1e6
                a[3] += 1
    n = len(pushes)
    print("pushes: %d, main-stream span %.3f ms per push" % (n, total / max(1, n)))
    print("%-28s %9s %9s %9s" % ("kernel", "start ms", "dur ms", "gap ms"))
    gaps = 0.0
    for name in order:
        a = acc[name]
        k = max(1, a[3])
        print("%-28s %9.3f %9.3f %9.3f%s" % (name, a[0] / k, a[1] / k, a[2] / k, "  (side stream)" if name in SIDE else ""))
        if name not in SIDE:
            gaps += a[2] / k
    print("sum of gaps on the main stream: %.3f ms per push" % gaps)


if __name__ == "__main__":
    main()
