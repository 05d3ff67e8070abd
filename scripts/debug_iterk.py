"""Find the first PH iteration where phx_iterk and the host loop differ (straggler case)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import mpisppy_amd  # noqa
from helpers import run_engine  # noqa
from mpisppy_amd.examples import farmer  # noqa

S = int(os.environ.get("S", "2000"))
so = {"as_rounds": int(os.environ.get("AS", "0")), "ipm_max_it": int(os.environ.get("IPM", "2"))}
for K in range(1, 5):
    res = []
    for nl in (1, 0):
        o = dict(so, native_loop=nl, iterk_depth=int(os.environ.get("DEPTH", "4")))
        ph, conv, Eobj, tb = run_engine(farmer.scenario_creator, farmer.scenario_names_creator(S), {"num_scens": S},
                                        K, options={"iter0_solver_options": dict(so), "iterk_solver_options": o})
        res.append((ph.W_array(), ph.nonant_values(), conv, getattr(ph, "iterk_stats", None),
                    [s.get("stragglers") for s in ph.solve_stats]))
    (Wa, xa, ca, sa, ta), (Wb, xb, cb, sb, tb_) = res
    dW = np.abs(Wa - Wb).max()
    dx = np.abs(xa - xb).max()
    bad = np.nonzero(np.abs(xa - xb).max(1) > 1e-9)[0]
    print("K=%d dW=%.3e dx=%.3e conv %r %r native %s host stragglers %s bad lanes %d %s" % (
        K, dW, dx, ca, cb, sa, tb_, len(bad), bad[:10]), flush=True)
