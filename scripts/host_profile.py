"""Host-side cost of one PH step on the GPU (farmer 100k): per-call wall times
(no device sync inside the step) and a cProfile of the Python path."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mpisppy_amd  # noqa: E402,F401
from mpisppy_amd.opt.ph import PH  # noqa: E402
from mpisppy_amd.examples import farmer  # noqa: E402

S = int(os.environ.get("SCENS", "100000"))
so = {"lane_solver": 1}
opts = {"solver_name": "phx", "PHIterLimit": 10 ** 9, "defaultPHrho": 1.0, "convthresh": 1e-10, "verbose": False,
        "display_progress": False, "iter0_solver_options": dict(so), "iterk_solver_options": dict(so)}
ph = PH(opts, farmer.scenario_names_creator(S), farmer.scenario_creator, scenario_creator_kwargs={"num_scens": S})
ph.PH_Prep()
ph.subproblem_creation(False)
ph.Iter0()
T = {"xbar": 0.0, "update_w": 0.0, "conv": 0.0, "solve": 0.0}


def step(timed):
    t0 = time.perf_counter()
    ph.Compute_Xbar(False)
    t1 = time.perf_counter()
    ph.Update_W(False)
    t2 = time.perf_counter()
    ph.conv = ph.convergence_diff()
    t3 = time.perf_counter()
    ph.solve_loop(solver_options=ph.current_solver_options, gripe=False)
    t4 = time.perf_counter()
    if timed:
        T["xbar"] += t1 - t0
        T["update_w"] += t2 - t1
        T["conv"] += t3 - t2
        T["solve"] += t4 - t3


for _ in range(20):
    step(False)
ph._settle()
torch.cuda.synchronize()
K = 500
t0 = time.perf_counter()
for _ in range(K):
    step(True)
ph._settle()
torch.cuda.synchronize()
dt = time.perf_counter() - t0
print("us/step %.1f" % (dt / K * 1e6), {k: round(v / K * 1e6, 1) for k, v in T.items()})
pr = cProfile.Profile()
pr.enable()
for _ in range(K):
    step(False)
ph._settle()
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(30)
