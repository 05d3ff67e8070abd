"""First PH iteration where phx_iterk's workgroup mode and the host loop differ
(farmer crops_multiplier=10), with the device loop's statistics."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import mpisppy_amd  # noqa
from helpers import run_engine  # noqa
from mpisppy_amd.examples import farmer  # noqa

S = int(os.environ.get("S", "1000"))
for K in range(1, 5):
    res = []
    for nl in (1, 0):
        so = {"native_loop": nl, "iterk_depth": int(os.environ.get("DEPTH", "4"))}
        ph, conv, Eobj, tb = run_engine(farmer.scenario_creator, farmer.scenario_names_creator(S),
                                        {"num_scens": S, "crops_multiplier": 10}, K,
                                        options={"iter0_solver_options": {}, "iterk_solver_options": so})
        res.append((ph.W_array(), ph.nonant_values(), conv, getattr(ph, "iterk_stats", None)))
    (Wa, xa, ca, sa), (Wb, xb, cb, _) = res
    print("K=%d dW=%.3e dx=%.3e conv %r %r stats %s" % (K, np.abs(Wa - Wb).max(), np.abs(xa - xb).max(), ca, cb, sa),
          flush=True)
