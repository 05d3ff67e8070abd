"""Probe: netdes network-50-30-H-01 LP relaxation (C5b: n = 2,940, m = 1,520, 1,470
nonants) through the engine on the GPU (generic PDHG + polish path).  Prints each
solve's stats and the trivial bound against the LP value HiGHS gives on the CPU
(75593.51224584531 for the 30 shipped scenarios, computed with oracle.qp.highs_solve)."""
import sys
import threading
import time

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
from helpers import rel, run_engine  # noqa: E402
from mpisppy_amd import _native  # noqa: E402
from mpisppy_amd.examples import netdes  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 30
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 2
lib = _native.load()
names = netdes.scenario_names_creator(S)
kw = {"instance": "network-50-30-H-01"}
if S != 30:
    kw["num_scens"] = S
solver = {}
if len(sys.argv) > 3:                      # pdhg_max_iters, polish
    solver = {"pdhg_max_iters": int(sys.argv[3]), "polish": int(sys.argv[4])}
if len(sys.argv) > 5:                      # ipm_after
    solver["ipm_after"] = int(sys.argv[5])
t = time.time()


def _beat():
    while True:
        time.sleep(30)
        print("... %.0f s" % (time.time() - t), flush=True)


threading.Thread(target=_beat, daemon=True).start()
ph, conv, Eobj, tb = run_engine(netdes.scenario_creator, names, kw, iters, lib=lib,
                                options={"iter0_solver_options": solver, "iterk_solver_options": solver})
print("S", S, "iters", iters, "wall %.2f s" % (time.time() - t), "tb %.10g" % tb, "conv", conv, flush=True)
if S == 30:
    print("trivial bound rel err vs HiGHS", rel(tb, 75593.51224584531))
for s in ph.solve_stats:
    print({k: v for k, v in s.items()})
