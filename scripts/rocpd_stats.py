"""Per-kernel duration statistics from a rocprofv3 run_results.db (rocpd SQLite
output), optionally over the last N launches of each kernel (a bench run's
timed window when it ends with its timed iterations).

    python scripts/rocpd_stats.py gpurun_out/<tag> [--last N] > profiles/<round>_<tag>_stats.txt
"""
import collections
import glob
import os
import sqlite3
import sys


def main(d, last=None):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*results.db"), recursive=True):
        con = sqlite3.connect(f)
        rows += con.execute("select name, dispatch_id, duration from kernels").fetchall()
    per = collections.defaultdict(list)
    for name, disp, dur in sorted(rows, key=lambda r: r[1]):
        per[name.split("(")[0]].append(dur / 1e3)
    print("%-34s %7s %11s %9s %9s %9s" % ("kernel", "calls", "total_us", "avg_us", "min_us", "max_us"))
    for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        if last:
            v = v[-last:]
        print("%-34s %7d %11.1f %9.2f %9.2f %9.2f" % (k[:34], len(v), sum(v), sum(v) / len(v), min(v), max(v)))


if __name__ == "__main__":
    a = sys.argv[1:]
    last = None
    if "--last" in a:
        i = a.index("--last")
        last = int(a[i + 1])
        del a[i:i + 2]
    main(a[0], last)
