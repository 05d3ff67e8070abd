"""Host-side time marks inside bench.py's timed run (Iter0 + K iterations) on
the GPU: where the Python between the device work goes.  Wraps the PHBase
methods the timed run calls and prints each one's wall time (median of R runs).

    python scripts/host_marks.py [S=100000] [K=20] [R=5]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.argv = [sys.argv[0]] + sys.argv[1:]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import bench  # noqa: E402
from mpisppy_amd import phbase, spopt, spbase  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
R = int(sys.argv[3]) if len(sys.argv) > 3 else 5
marks = {}


def wrap(cls, name):
    f = getattr(cls, name)

    def w(self, *a, **k):
        t = time.perf_counter()
        try:
            return f(self, *a, **k)
        finally:
            marks.setdefault(cls.__name__ + "." + name, []).append(time.perf_counter() - t)
    setattr(cls, name, w)


for cls, names in [(phbase.PHBase, ["Iter0", "iterk_loop", "_iterk_native", "_resolve_deferred_iter0",
                                    "_iterk_finish", "_iter0_deferred_start", "_record_solve"]),
                   (spopt.SPOpt, ["solve_loop", "_set_ph_terms", "_save_original_nonants", "_create_solvers"]),
                   (spbase.SPBase, ["_settle", "_check_stream"])]:
    for n in names:
        if hasattr(cls, n):
            wrap(cls, n)

torch.cuda.set_device(0)
dev = bench.Dev("cuda")
W = bench.workloads()
so = {"lane_solver": 1, "iterk_depth": 4, "iterk_timing": 5, "iterk_fused": 1}
lib_iterk = None
tot = []
for r in range(R + 1):
    ph = bench.make_ph(W["C3"], S, 1, 1.0, so, K, dev)
    torch.cuda.synchronize()
    marks.clear()
    # the native call itself
    nat = ph._native
    orig = nat.iterk
    tk = []

    def it(*a, _o=orig):
        t = time.perf_counter()
        rr = _o(*a)
        tk.append(time.perf_counter() - t)
        return rr
    nat.iterk = it
    T = bench.timed_run(ph, K, dev)
    nat.iterk = orig
    if r == 0:
        continue
    tot.append((T, dict((k, sum(v)) for k, v in marks.items()), sum(tk)))
    del ph
print("S=%d K=%d, median over %d runs (us):" % (S, K, R))
print("  T %.1f  Iter0(events) %.1f" % (np.median([t[0][0] for t in tot]) * 1e6, np.median([t[0][1] for t in tot]) * 1e6))
print("  lib.iterk (C call) %.1f" % (np.median([t[2] for t in tot]) * 1e6))
for k in sorted(tot[0][1]):
    print("  %-40s %8.1f" % (k, np.median([t[1].get(k, 0.0) for t in tot]) * 1e6))
