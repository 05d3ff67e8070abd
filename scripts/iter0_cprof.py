"""Host-side anatomy of the bench's timed region (Iter0 + K iterations, farmer
100k on the GPU): wall times of Iter0 pieces and a cProfile of the second run."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from mpisppy_amd.examples import farmer  # noqa: E402

S = int(os.environ.get("SCENS", "100000"))
w = {"names": farmer.scenario_names_creator, "creator": farmer.scenario_creator,
     "kw": lambda S, cm: {"num_scens": S, "crops_multiplier": cm}, "nodes": None}
ph = bench.make_ph(w, S, 1, 1.0, {}, 20)
print("warm", bench.timed_run(ph, 20))
pr = cProfile.Profile()
pr.enable()
t = bench.timed_run(ph, 20)
pr.disable()
print("timed", t)
st = pstats.Stats(pr)
rows = sorted(st.stats.items(), key=lambda kv: -kv[1][3])
print("%10s %10s %6s  %s" % ("cum_us", "tot_us", "calls", "function"))
for (f, ln, fn), (cc, nc, tt, ct, callers) in rows[:60]:
    print("%10.1f %10.1f %6d  %s:%d(%s)" % (ct * 1e6, tt * 1e6, nc, os.path.basename(f), ln, fn))
