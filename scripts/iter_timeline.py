"""Kernel timeline of the LAST timed Iter0 + loop in a rocprofv3 --kernel-trace
database (bench.py's timed run: the last k_seed_lanes / first-solve launch on).

    python scripts/iter_timeline.py gpurun_out/<tag>/run_results.db [first-kernel-substring]
"""
import sqlite3
import sys

db = sys.argv[1]
first = sys.argv[2] if len(sys.argv) > 2 else None
c = sqlite3.connect(db)
ks = [(s, e, n.split("(")[0][:34]) for n, s, e in c.execute("select name,start,end from kernels order by start")]
cp = [(s, e, "copy %d B" % z) for s, e, z in c.execute("select start,end,size from memory_copies")]
starts = [i for i, k in enumerate(ks) if (first in k[2] if first else k[2] in ("k_seed_lanes",))]
if not starts:
    starts = [i for i, k in enumerate(ks) if k[2] == "phx_lane_cold"]
    # the timed run's first solve: the second-to-last group of cold launches over all lanes
i0 = starts[-1]
t0 = ks[i0][0]
ev = sorted([x for x in ks + cp if x[0] >= t0])
prev = None
tot = {}
for s, e, n in ev:
    print("%-36s %9.1f %8.1f %8.1f" % (n, (s - t0) / 1e3, (e - s) / 1e3, (s - prev) / 1e3 if prev else 0.0))
    prev = e
