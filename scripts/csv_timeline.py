"""Kernel timeline of a rocprofv3 --kernel-trace CSV: every dispatch from the
N-th launch of a kernel on, start relative to it, duration and the gap to the
previous kernel's end (us).  python scripts/csv_timeline.py <run_kernel_trace.csv> <kernel> <nth> <count>"""
import csv
import sys

path, kname, nth, count = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:40])
        for r in csv.DictReader(open(path))]
rows.sort()
ks = [i for i, x in enumerate(rows) if x[2].startswith(kname)]
i0 = ks[nth]
t0 = rows[i0][0]
prev = None
for s, e, n in rows[i0:i0 + count]:
    print("%-42s %9.1f %8.1f %7.1f" % (n, (s - t0) / 1e3, (e - s) / 1e3, (s - prev) / 1e3 if prev else 0.0))
    prev = e
