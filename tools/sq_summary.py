#!/usr/bin/env python3
"""Per-kernel averages of the SQ counter passes written by tools/pmc_sq.sh.
Usage: python3 tools/sq_summary.py gpurun_out/sq_<tag> [kernel ...]"""
import glob
import os
import sqlite3
import sys
from collections import defaultdict


def short(name):
    return name.split("(")[0].replace("void ", "").replace("fvad::", "").split("<")[0]


def main():
    d = sys.argv[1]
    want = set(sys.argv[2:])
    vals = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, "**", "*.db"), recursive=True)):
        c = sqlite3.connect(f)
        for name, ctr, val in c.execute("select kernel_name, counter_name, value from counters_collection"):
            k = short(name)
            if not want or k in want:
                vals[k][ctr].append(float(val))
    for k in sorted(vals):
        print(k)
        for ctr in sorted(vals[k]):
            v = vals[k][ctr]
            v = v[1:] if len(v) > 1 else v
            print("  %-24s %16.1f" % (ctr, sum(v) / len(v)))


if __name__ == "__main__":
    main()
