"""Oracle PH trajectories for the full-trajectory parity tests of the larger sparse
configs (tests/test_trajectories.py): netdes network-50-30-H (C5b) on its 30 shipped
scenarios and sslp_15_45 (C5a) on 256 synthetic scenarios.

Both have degenerate Iter0 LPs (several optimal vertices), so a trajectory is pinned
from a given Iter0 point: the fixture holds the oracle's Iter0 nonants, and the engine
test overwrites its own Iter0 nonants with them before its PH iterations; from
iteration 1 on the prox term makes each subproblem's nonant optimum unique, so the
engine's W / x-bar / conv / nonants must follow the oracle's trajectory.

The oracle (test infrastructure: numpy PH loop + scipy-HiGHS + certified polish, or
its sparse interior point) takes ~1 s per netdes-50 QP on one core, too slow for
the GPU box's test budget; the trajectories are computed here once and committed as
.npz data (inputs + expected outputs, nothing executable).

    python tests/golden/make_trajectories.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

CASES = {
    "netdes50_30": dict(K=3),
    "sslp_256": dict(K=3),
}


def scens_of(case):
    from oracle import models as om
    if case == "netdes50_30":
        return [om.netdes("Scenario%d" % k, "network-50-30-H-01") for k in range(30)]
    if case == "sslp_256":
        return [om.sslp("Scenario%d" % k, num_scens=256) for k in range(1, 257)]
    raise KeyError(case)


def make(case):
    from oracle import ph as oph
    K = CASES[case]["K"]
    o = oph.OraclePH(scens_of(case), rho=1.0)
    tb = o.iter0()
    x0n = o.xn().copy()
    xbars, xsqbars, convs = [], [], []
    for _ in range(K):
        o.compute_xbar()
        o.update_w()
        convs.append(o.convergence_diff())
        xbars.append(o.xbar[0].copy())
        xsqbars.append(o.xsqbar[0].copy())
        o.solve_loop()
    out = os.path.join(HERE, "traj_%s.npz" % case)
    np.savez_compressed(out, K=K, rho=1.0, trivial_bound=tb, x0n=x0n, xbar=np.array(xbars),
                        xsqbar=np.array(xsqbars), conv=np.array(convs), W=o.W, xn=o.xn(), obj=o.obj)
    print("wrote", out, os.path.getsize(out), "bytes")


if __name__ == "__main__":
    for c in (sys.argv[1:] or CASES):
        make(c)
