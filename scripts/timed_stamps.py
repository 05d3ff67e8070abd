"""Host wall-clock stamps inside bench.py's timed region (farmer 100k, Iter0 + K
PH iterations, the collector off as in bench.timed_run): where the host time
before the first launch and after the device drain goes.  Medians over R runs.

    python scripts/timed_stamps.py [S=100000] [K=20] [R=7]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import bench  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
R = int(sys.argv[3]) if len(sys.argv) > 3 else 7
torch.cuda.set_device(0)
dev = bench.Dev("cuda")
W = bench.workloads()
so = {"lane_solver": 1, "iterk_depth": 4, "iterk_timing": 0, "iterk_fused": 1}
rows = []
for r in range(R + 1):
    ph = bench.make_ph(W["C3"], S, 1, 1.0, so, K, dev)
    bench.gc_settle()
    warm = bench.make_ph(W["C3"], S, 1, 1.0, so, 3, dev)
    warm.ph_main(finalize=False)
    dev.sync()
    del warm
    st = {}
    nat = ph._native
    orig_iterk, orig_solve = nat.iterk, nat.solve

    def iterk(*a, _o=orig_iterk):
        st["c_in"] = time.perf_counter()
        rr = _o(*a)
        st["c_out"] = time.perf_counter()
        return rr

    def solve(*a, _o=orig_solve):
        st.setdefault("solve_in", time.perf_counter())
        rr = _o(*a)
        st.setdefault("solve_out", time.perf_counter())
        return rr
    nat.iterk, nat.solve = iterk, solve
    ph.PH_Prep()
    ph.subproblem_creation(False)
    ph.options["PHIterLimit"] = K
    with bench.no_gc():
        dev.sync()
        t0 = time.perf_counter()
        ph._defer_iter0_checks = True
        ph.Iter0()
        st["iter0_out"] = time.perf_counter()
        ph.iterk_loop()
        st["iterk_out"] = time.perf_counter()
        ph._settle()
        st["settle_out"] = time.perf_counter()
        dev.sync()
        st["sync_out"] = time.perf_counter()
    nat.iterk, nat.solve = orig_iterk, orig_solve
    if r:
        rows.append({k: (v - t0) * 1e6 for k, v in st.items()})
    del ph
keys = ["solve_in", "solve_out", "iter0_out", "c_in", "c_out", "iterk_out", "settle_out", "sync_out"]
print("S=%d K=%d: host stamps from t0, median over %d runs (us)" % (S, K, R))
for k in keys:
    print("  %-11s %8.1f" % (k, np.median([rw[k] for rw in rows if k in rw])))
