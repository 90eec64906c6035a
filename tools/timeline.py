#!/usr/bin/env python3
"""Per-push GPU timeline from a rocprofv3 --kernel-trace --memory-copy-trace
run of bench.py (sqlite output): every kernel / copy of the last pushes with
its queue and the idle gap before it on the main queue (diagnostic).
Usage: python3 tools/timeline.py <rocprofv3 output dir> [n_rows]"""
import glob
import os
import sqlite3
import sys


def main():
    d = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
        c = sqlite3.connect(f)
        for s, e, name, q in c.execute("select start, end, name, queue_id from kernels"):
            rows.append((s, e, name.split("(")[0].replace("void ", "")[:44], q))
        for s, e, name, q in c.execute("select start, end, name, queue_id from memory_copies"):
            rows.append((s, e, "COPY " + str(name)[:38], q))
    rows.sort()
    rows = rows[-n:]
    t0 = rows[0][0]
    busy_until = rows[0][0]
    for s, e, name, q in rows:
        gap = max(0, s - busy_until)
        print("%9.1f us  dur %8.1f  idle-before %6.1f  q%-3s %s" % ((s - t0) / 1e3, (e - s) / 1e3, gap / 1e3, q, name))
        busy_until = max(busy_until, e)


if __name__ == "__main__":
    main()
