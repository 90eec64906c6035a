#!/usr/bin/env python3
"""Summarise a tools/profile.sh run into profiles/.

- profiles/<tag>_kernel_stats.csv : rocprofv3 --stats summary (trace pass)
- profiles/pmc_traffic[_<mode>].json : per-kernel HBM bytes per launch from the
  FETCH_SIZE and WRITE_SIZE passes (kilobytes in rocprofv3), corrected as
  MI355X_MICROARCH.md prescribes for gfx950: FETCH_SIZE counts 128-B memory
  requests at 64 B, so it is doubled; WRITE_SIZE is taken as is.
bench.py reads pmc_traffic.json for roofline.traffic when its workload
(streams, ticks, channels, mode) matches.
"""
import csv
import glob
import json
import os
import shutil
import sqlite3
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    n = name.split("(")[0]
    n = n.replace("void ", "").replace("fvad::", "")
    return n.split("<")[0]


def counters(d, counter):
    """Per-kernel list of per-dispatch counter values (rocpd .db or csv output)."""
    per = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(d, "**", "*.db"), recursive=True)):
        c = sqlite3.connect(f)
        for name, val in c.execute("select kernel_name, value from counters_collection where counter_name = ? "
                                   "order by dispatch_id", (counter,)):
            per[short(name)].append(float(val))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") == counter:
                    per[short(row["Kernel_Name"])].append(float(row["Counter_Value"]))
    return per


def write_stats(d, dst):
    """--stats summary as csv (Name, Calls, TotalDurationNs, AverageNs, Percentage)."""
    for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
        shutil.copy(f, dst)
        return True
    for f in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
        c = sqlite3.connect(f)
        rows = list(c.execute("select name, total_calls, total_duration, average, percentage from top_kernels"))
        # rocpd top_kernels durations are in microseconds
        with open(dst, "w", newline="") as fh:
            w = csv.writer(fh, quoting=csv.QUOTE_NONNUMERIC)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
            for name, calls, tot, avg, pct in rows:
                w.writerow([name, calls, round(tot * 1000.0), round(avg * 1000.0, 1), round(pct, 3)])
        return True
    return False


def main():
    out, tag = sys.argv[1], sys.argv[2]
    args = sys.argv[3:]
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    write_stats(os.path.join(out, "trace"), os.path.join(ROOT, "profiles", "%s_kernel_stats.csv" % tag))
    fetch = counters(os.path.join(out, "fetch"), "FETCH_SIZE")
    write = counters(os.path.join(out, "write"), "WRITE_SIZE")
    # bench.py's defaults; groups = engines per GPU (a launch covers streams / groups)
    cfg = {"streams": 2048, "ticks": 50, "channels": 2, "mode": "staged", "groups": 1}
    keys = {"--streams-per-gpu": "streams", "--ticks": "ticks", "--channels": "channels", "--mode": "mode",
            "--groups": "groups"}
    for i, a in enumerate(args):
        if a in keys and i + 1 < len(args):
            v = args[i + 1]
            cfg[keys[a]] = v if keys[a] == "mode" else int(v)
    res = dict(cfg)
    res["tag"] = tag
    res["correction"] = "FETCH_SIZE x2 (gfx950 128-B requests tallied at 64 B), WRITE_SIZE x1; KB -> bytes x1024"
    res["bytes_per_launch"] = {}
    res["fetch_kb_raw"] = {}
    res["write_kb_raw"] = {}
    for k in sorted(set(fetch) | set(write)):
        # skip the first (warm-up/cold) dispatch when there are several
        f = fetch.get(k, [0.0])
        w = write.get(k, [0.0])
        f = f[1:] if len(f) > 1 else f
        w = w[1:] if len(w) > 1 else w
        fa, wa = sum(f) / len(f), sum(w) / len(w)
        res["fetch_kb_raw"][k] = fa
        res["write_kb_raw"][k] = wa
        res["bytes_per_launch"][k] = (2 * fa + wa) * 1024.0
    name = "pmc_traffic.json" if cfg["mode"] == "staged" else "pmc_traffic_%s.json" % cfg["mode"]
    with open(os.path.join(ROOT, "profiles", name), "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
