"""Host launch time against device start, per dispatch, from a rocprofv3
--kernel-trace --hip-runtime-trace run: for every kernel from the N-th launch
of <kernel> on, its start / duration / gap to the previous kernel's end (us,
as csv_timeline.py) and when the host made the launch call, relative to the
kernel's start (negative: enqueued ahead; near zero or positive gap: the
device waited for the host).
python scripts/launch_lag.py <dir with run_kernel_trace.csv, run_hip_api_trace.csv> <kernel> <nth> <count>"""
import csv
import os
import sys

d, kname, nth, count = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
api = {}
for r in csv.DictReader(open(os.path.join(d, "run_hip_api_trace.csv"))):
    api[r["Correlation_Id"]] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"])
rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:34],
               r["Correlation_Id"]) for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))))
ks = [i for i, x in enumerate(rows) if x[2].startswith(kname)]
i0 = ks[nth]
t0 = rows[i0][0]
prev = None
print("%-34s %9s %8s %7s %9s %7s  %s" % ("kernel", "start", "dur", "gap", "call-st", "call", "api"))
for s, e, n, c in rows[i0:i0 + count]:
    a = api.get(c)
    cs, cd, fn = ((a[0] - s) / 1e3, (a[1] - a[0]) / 1e3, a[2]) if a else (float("nan"), float("nan"), "?")
    print("%-34s %9.1f %8.1f %7.1f %9.1f %7.1f  %s" % (n, (s - t0) / 1e3, (e - s) / 1e3,
                                                       (s - prev) / 1e3 if prev else 0.0, cs, cd, fn))
    prev = e
