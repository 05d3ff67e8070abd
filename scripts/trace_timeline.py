"""Merged timeline (host HIP API calls + kernels + copies) of a rocprofv3
--kernel-trace --hip-runtime-trace run around the N-th launch of a kernel.

    python scripts/trace_timeline.py gpurun_out/<tag> <kernel> <nth> <count>
"""
import glob
import sqlite3
import sys

d, kname, nth, count = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
f = glob.glob(d + "/**/*.db", recursive=True)[0]
c = sqlite3.connect(f)
ev = [(s, e, "K " + n.split("(")[0][:40]) for n, s, e in c.execute("select name,start,end from kernels")]
ev += [(s, e, "C %d B" % sz) for s, e, sz in c.execute("select start,end,size from memory_copies")]
ev += [(s, e, "  api " + n[:40]) for n, s, e in c.execute("select name,start,end from regions")
       if not n.startswith(("hipGetLastError", "hipGetDevice", "hipSetDevice", "hipPeekAtLastError"))]
ev.sort()
ks = [i for i, x in enumerate(ev) if x[2].startswith("K " + kname)]
i0 = ks[nth]
t0 = ev[i0][0]
for s, e, n in ev[i0 - 5:i0 - 5 + count]:
    print("%-48s %10.1f %8.1f" % (n, (s - t0) / 1e3, (e - s) / 1e3))
