"""Host-side cProfile of bench.py's timed region (Iter0 + K PH iterations,
farmer 100k by default): where the wall time between kernels goes.

    python scripts/timed_profile.py [K] > gpurun_out/timed_profile.txt
"""
import cProfile
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import mpisppy_amd  # noqa: E402,F401

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
S = int(os.environ.get("SCENS", "100000"))
torch.cuda.set_device(0)
W = bench.workloads()["C3"]
so = {"lane_solver": 1, "iterk_depth": 4, "iterk_timing": 5, "iterk_fused": 1}
ph = bench.make_ph(W, S, 1, 1.0, so, 3)
ph.ph_main(finalize=False)
torch.cuda.synchronize()
for rep in range(2):
    ph = bench.make_ph(W, S, 1, 1.0, so, K)
    torch.cuda.synchronize()
    pr = cProfile.Profile() if rep == 1 else None
    if pr:
        pr.enable()
    T, T0, Tk = bench.timed_run(ph, K)
    if pr:
        pr.disable()
    print("rep %d: T %.3f ms  Iter0 %.3f ms  iterk %.3f ms" % (rep, T * 1e3, T0 * 1e3, Tk * 1e3))
print("Iter0 solve stats:", ph.solve_stats[0])
print("iterk stats:", getattr(ph, "iterk_stats", None))
st = pstats.Stats(pr)
st.sort_stats("cumulative").print_stats(45)
st.sort_stats("tottime").print_stats(25)
