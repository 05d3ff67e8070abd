"""Host cost of the bench's timed region (farmer 100k, Iter0 + 20 iterations):
wall stamps around Iter0 / iterk_loop / _settle / the device sync, and a
cProfile of one timed run (the second of three), sorted by own time.
python scripts/timed_cprof.py  (GPU box)"""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import mpisppy_amd  # noqa: E402,F401
from mpisppy_amd.examples import farmer  # noqa: E402
import torch  # noqa: E402

S = int(os.environ.get("SCENS", "100000"))
w = {"names": farmer.scenario_names_creator, "creator": farmer.scenario_creator,
     "kw": lambda S, cm: {"num_scens": S, "crops_multiplier": cm}, "nodes": None}
dev = bench.Dev("cuda")


def stamped(ph, K):
    ph.PH_Prep()
    ph.subproblem_creation(False)
    ph.options["PHIterLimit"] = K
    ph.mpicomm.Barrier()
    torch.cuda.synchronize()
    t = [time.perf_counter()]
    ph._defer_iter0_checks = True
    ph.Iter0()
    t.append(time.perf_counter())
    ph.iterk_loop()
    t.append(time.perf_counter())
    ph._settle()
    t.append(time.perf_counter())
    torch.cuda.synchronize()
    t.append(time.perf_counter())
    ph.mpicomm.Barrier()
    t.append(time.perf_counter())
    st = ph.iterk_stats
    return [(b - a) * 1e6 for a, b in zip(t[:-1], t[1:])], (t[-1] - t[0]) * 1e6, st["wall_s"] * 1e6


for rep in range(4):
    ph = bench.make_ph(w, S, 1, 1.0, {}, 20, dev)
    torch.cuda.synchronize()
    if rep == 2:
        pr = cProfile.Profile()
        pr.enable()
    parts, tot, wall = stamped(ph, 20)
    if rep == 2:
        pr.disable()
    print("run %d: total %.1f us | Iter0 %.1f, iterk_loop %.1f (phx_iterk wall %.1f), _settle %.1f, sync %.1f, "
          "barrier %.1f" % (rep, tot, parts[0], parts[1], wall, parts[2], parts[3], parts[4]), flush=True)
    del ph
    torch.cuda.empty_cache()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
pstats.Stats(pr).sort_stats("cumulative").print_stats(30)
