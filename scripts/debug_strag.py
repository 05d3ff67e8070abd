"""Debug: native (phx_iterk, unfused) vs host PH loop (deferred / not deferred)
with starved lane solves: x-bar and W after ITERS iterations."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from helpers import run_engine  # noqa: E402
from mpisppy_amd import _native  # noqa: E402
from mpisppy_amd.examples import farmer  # noqa: E402

lib = _native.load()
solver = {"as_rounds": 1, "ipm_max_it": 3}
ITERS = int(sys.argv[1]) if len(sys.argv) > 1 else 3
runs = {}
for name, extra in [("native", {"native_loop": 1, "iterk_fused": 0}), ("host_defer", {"native_loop": 0}),
                    ("host_nodefer", {"native_loop": 0, "defer": 0})]:
    so = dict(solver, **extra)
    opts = {"iter0_solver_options": dict(solver), "iterk_solver_options": so}
    ph = run_engine(farmer.scenario_creator, farmer.scenario_names_creator(2000), {"num_scens": 2000}, ITERS,
                    lib=lib, device=None, options=opts)[0]
    runs[name] = ph
    print(name, "xbar", ph.xbar_by_node()["ROOT"][0], "mean x", ph.nonant_values().mean(axis=0),
          "strag", [s.get("stragglers") for s in ph.solve_stats])
for a in runs:
    for b in runs:
        if a < b:
            print(a, b, "W maxdiff", np.abs(runs[a].W_array() - runs[b].W_array()).max())
