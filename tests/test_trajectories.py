"""Full PH trajectories of the larger sparse configs against the oracle (north_star bar:
W 1e-6, x-bar 1e-8, every subproblem optimum 1e-6 in the nonants / 1e-8 in value):

* C5b netdes network-50-30-H on its 30 shipped scenarios (n = 2,940, m = 1,520,
  1,470 nonants: the sparse workgroup solver, phx_sp.h),
* C5a sslp_15_45 on 256 synthetic scenarios (n = 705, m = 60: the workgroup warm
  pass, phx_wg.h, through the device loop).

Their Iter0 LPs are degenerate, so the trajectory is pinned from a common Iter0
point: the engine runs its own Iter0 (the trivial bound, a unique LP value, must
match), then takes the oracle's Iter0 nonants (tests/golden/traj_*.npz, made by
tests/golden/make_trajectories.py) and runs K PH iterations; W, x-bar, x-sq-bar,
conv and the final subproblem optima must follow the oracle's trajectory
(phbase.py:27-107, 293-343, 875-979)."""
import os

import numpy as np
import pytest

from helpers import all_certified, ph_options, rel
from mpisppy_amd.examples import netdes, sslp
from mpisppy_amd.opt.ph import PH

HERE = os.path.dirname(os.path.abspath(__file__))


def _case(case):
    if case == "netdes50_30":
        return netdes.scenario_creator, netdes.scenario_names_creator(30), {"instance": "network-50-30-H-01"}
    if case == "sslp_256":
        return sslp.scenario_creator, sslp.scenario_names_creator(256), {"num_scens": 256}
    raise KeyError(case)


def check_trajectory(lib, device, case, solver=None):
    z = np.load(os.path.join(HERE, "golden", "traj_%s.npz" % case), allow_pickle=False)
    K = int(z["K"])
    creator, names, kw = _case(case)
    ph = PH(ph_options(K, rho=float(z["rho"]), solver=solver), names, creator, scenario_creator_kwargs=kw,
            _native_lib=lib, _device=device)
    ph.PH_Prep()
    ph.subproblem_creation(False)
    tb = ph.Iter0()
    assert rel(tb, float(z["trivial_bound"])) < 1e-9
    ph._set_nonant_x(z["x0n"])                 # the oracle's Iter0 vertex
    ph.iterk_loop()
    ph._settle()
    assert ph._PHIter == K and all_certified(ph)
    xb, xsq = ph.xbar_by_node()["ROOT"]
    assert rel(xb, z["xbar"][-1]) < 1e-8
    assert rel(xsq, z["xsqbar"][-1]) < 1e-8
    assert rel(ph.conv, z["conv"][-1]) < 1e-6
    assert rel(ph.W_array(), z["W"]) < 1e-6
    assert rel(ph.nonant_values(), z["xn"]) < 1e-6
    assert rel(ph._host("obj"), z["obj"]) < 1e-8
    return ph


def test_sslp_256_trajectory_emu(emu):
    check_trajectory(emu, "cpu", "sslp_256")


def test_netdes50_trajectory_emu(emu):
    check_trajectory(emu, "cpu", "netdes50_30")


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["sslp_256", "netdes50_30"])
def test_trajectory_gpu(gpu_lib, case):
    ph = check_trajectory(gpu_lib, None, case)
    if case == "sslp_256":
        assert hasattr(ph, "iterk_stats")       # the device loop (workgroup pass) ran the iterations
