"""Iter0 / first-iterations anatomy on the GPU (farmer, S scenarios): per solve
which lanes the warm / seeded passes certified, how many went to the cold
interior point and the generic path, wall times; variants by solver options.

    python scripts/iter0_probe.py S key=val ...   (iter0/iterk solver options)
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import mpisppy_amd  # noqa
from helpers import ph_options  # noqa
from mpisppy_amd.examples import farmer  # noqa
from mpisppy_amd.opt.ph import PH  # noqa

S = int(sys.argv[1])
so = {}
for kv in sys.argv[2:]:
    k, v = kv.split("=")
    so[k] = float(v) if "." in v or "e" in v else int(v)
for rep in range(2):
    opts = ph_options(3)
    opts["iter0_solver_options"] = dict(so)
    opts["iterk_solver_options"] = dict(so, native_loop=0)
    ph = PH(opts, farmer.scenario_names_creator(S), farmer.scenario_creator, scenario_creator_kwargs={"num_scens": S})
    ph.PH_Prep()
    ph.subproblem_creation(False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ph.Iter0()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    ph.iterk_loop()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("rep %d opts %s: Iter0 %.3f ms, 3 iterations %.3f ms" % (rep, so, 1e3 * (t1 - t0), 1e3 * (t2 - t1)))
    for k, st in enumerate(ph.solve_stats):
        print("  solve %d: %s" % (k, {kk: (round(v, 4) if isinstance(v, float) else v) for kk, v in st.items()}))
