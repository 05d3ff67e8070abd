"""Summarise a rocprofv3 --kernel-trace run (rocpd SQLite .db or kernel_stats.csv)
into the per-kernel stats CSV committed under profiles/.

    python scripts/prof_summary.py gpurun_out/prof5 > profiles/r01_xxx.csv
"""
import csv
import glob
import os
import sqlite3
import sys


def from_db(path):
    c = sqlite3.connect(path)
    rows = c.execute("select name, count(*), sum(duration), avg(duration) from kernels group by name").fetchall()
    tot = sum(r[2] for r in rows) or 1
    return [(n.split("(")[0], k, s / 1e3, a / 1e3, 100.0 * s / tot) for n, k, s, a in rows]


def from_csv(path):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            out.append((r["Name"].split("(")[0], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3,
                        float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
    return out


def main(d):
    dbs = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)
    csvs = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    rows = from_db(dbs[0]) if dbs else from_csv(csvs[0])
    rows.sort(key=lambda r: -r[2])
    print("name,total_calls,total_duration_us,average_us,percentage")
    for n, k, s, a, p in rows:
        print('"%s",%d,%.3f,%.3f,%.4f' % (n[:120], k, s, a, p))


if __name__ == "__main__":
    main(sys.argv[1])
