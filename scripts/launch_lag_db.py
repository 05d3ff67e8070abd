"""launch_lag.py for rocprofv3's default sqlite output (run_results.db):
per dispatch from the N-th launch of <kernel>: start, duration, gap to the
previous kernel's end, and the host launch call's start relative to the
kernel's start (us).  python scripts/launch_lag_db.py <run_results.db> <kernel> <nth> <count>"""
import sqlite3
import sys

db, kname, nth, count = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
c = sqlite3.connect(db)
reg = {sid: (s, e, n) for sid, s, e, n in c.execute("select stack_id, start, end, name from regions")}
rows = list(c.execute("select start, end, name, stack_id from kernels order by start"))
ks = [i for i, r in enumerate(rows) if r[2].startswith(kname)]
i0 = ks[nth]
t0 = rows[i0][0]
prev = None
print("%-34s %9s %8s %7s %9s %7s  %s" % ("kernel", "start", "dur", "gap", "call-st", "call", "api"))
for s, e, n, sid in rows[i0:i0 + count]:
    a = reg.get(sid)
    cs, cd, fn = ((a[0] - s) / 1e3, (a[1] - a[0]) / 1e3, a[2]) if a else (float("nan"), float("nan"), "?")
    print("%-34s %9.1f %8.1f %7.1f %9.1f %7.1f  %s" % (n.split("(")[0][:34], (s - t0) / 1e3, (e - s) / 1e3,
                                                       (s - prev) / 1e3 if prev else 0.0, cs, cd, fn))
    prev = e
