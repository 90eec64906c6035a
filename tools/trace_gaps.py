"""Push timeline from a rocprofv3 kernel-trace database (a rocprofv3 --kernel-trace run of bench.py, e.g. tools/profile.sh):
per-boundary gaps of the main-stream chain, push period, main-chain busy
time, and what the side kernels overlap.  Usage: trace_gaps.py <run_results.db>"""
import collections
import re
import sqlite3
import sys

MAIN = ["k_fftAw", "k_plpc", "k_pcorr", "k_select", "k_pspecw", "k_rnn3", "k_gru16", "k_synthw", "k_olafb"]


def main(db):
    c = sqlite3.connect(db)
    sym = {r[0]: r[1] for r in c.execute("select id, kernel_name from rocpd_info_kernel_symbol")}

    def nm(s):
        m = re.search(r"(k_[A-Za-z0-9_]+?)E", s)
        return m.group(1) if m else s
    rows = [(nm(sym[k]), s, e) for k, s, e in c.execute("select kernel_id, start, end from rocpd_kernel_dispatch order by start")]
    mc = [x for x in rows if x[0] in MAIN]
    gaps = collections.defaultdict(list)
    for a, b in zip(mc, mc[1:]):
        gaps[(a[0], b[0])].append((b[1] - a[2]) / 1000)
    for k, v in gaps.items():
        v = sorted(v)
        print("%-24s median %7.2f us  max %8.2f" % ("%s->%s" % k, v[len(v) // 2], v[-1]))
    st = [x[1] for x in mc if x[0] == "k_fftAw"]
    per = sorted((b - a) / 1e6 for a, b in zip(st, st[1:]))
    busy = sorted(sum(x[2] - x[1] for x in mc if s0 <= x[1] < s1) / 1e6 for s0, s1 in zip(st, st[1:]))
    print("push period ms: median %.3f (min %.3f)  main busy median %.3f" % (per[len(per) // 2], per[0], busy[len(busy) // 2]))
    dur = collections.defaultdict(list)
    for n, s, e in rows:
        dur[n].append((e - s) / 1e6)
    print({k: round(sorted(v)[len(v) // 2], 3) for k, v in dur.items()})


if __name__ == "__main__":
    main(sys.argv[1])
