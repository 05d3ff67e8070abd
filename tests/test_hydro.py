"""hydro (three-stage LP, BF [3,3]) through the engine: the reference's only multistage
PH pin (test_ef_ph.py:622-640: trivial bound 180, Eobjective with W and prox disabled
190, 2 sig), and engine == oracle on the whole PH run (per-node conditional x-bar with
prob_coeff 1/9 at ROOT and 1/3 at ROOT_b, W of both stages) at the north_star bar."""
import numpy as np
import pytest

from helpers import all_certified, oracle_continue_from, rel, run_engine
from mpisppy_amd.examples import hydro
from mpisppy_amd.utils import sputils
from oracle import models as om
from test_oracle_golden import G, hydro_oracle_ph, round_pos_sig

BFS = [3, 3]


def test_hydro_model_matches_oracle():
    for nm in ["Scen1", "Scen5", "Scen9"]:
        sf = hydro.scenario_creator(nm, branching_factors=BFS).standard_form()
        o = om.hydro(nm, BFS)
        # same LP up to the column order: compare through variable names
        names = [v.name for v in hydro.scenario_creator(nm, branching_factors=BFS)._vars]
        perm = [names.index(v) for v in o.var_names]
        A = np.zeros((len(sf["bl"]), len(names)))
        for i in range(len(sf["bl"])):
            for k in range(sf["rowptr"][i], sf["rowptr"][i + 1]):
                A[i, sf["colidx"][k]] = sf["vals"][k]
        assert np.allclose(A[:, perm], o.A, rtol=1e-15, atol=0)
        assert np.allclose(sf["bl"], o.bl, rtol=1e-15) and np.allclose(sf["bu"], o.bu, rtol=1e-15)
        assert np.array_equal(sf["lb"][perm], o.lb) and np.array_equal(sf["ub"][perm], o.ub)
        assert np.array_equal(sf["c"][perm], o.c)


def check_hydro(lib, device, native_loop=1):
    g = G["hydro_ph_bf33"]
    names = hydro.scenario_names_creator(9)
    so = {"native_loop": native_loop}
    ph, conv, Eobj, tb = run_engine(hydro.scenario_creator, names, {"branching_factors": BFS}, g["PHIterLimit"],
                                    rho=g["rho"], lib=lib, device=device,
                                    all_nodenames=sputils.create_nodenames_from_branching_factors(BFS),
                                    options={"convthresh": g["convthresh"], "iter0_solver_options": so,
                                             "iterk_solver_options": so})
    assert all_certified(ph)
    ph.disable_W_and_prox()
    E_nowp = ph.Eobjective()
    # the reference's asserts (2 significant digits)
    assert round_pos_sig(tb, g["sig"]) == g["trivial_bound"]
    assert round_pos_sig(E_nowp, g["sig"]) == g["Eobj_W_prox_disabled"]
    # the oracle's run: Iter0 optimum values equal; hydro's Iter0 LPs are degenerate
    # (several optimal vertices), so the oracle's PH iterations start from the
    # engine's Iter0 point (from iteration 1 on the prox term makes each nonant
    # optimum unique) and the two trajectories must agree
    o, oconv, oE, otb, oE_nowp = hydro_oracle_ph()
    assert rel(tb, otb) < 1e-9
    ph0 = run_engine(hydro.scenario_creator, names, {"branching_factors": BFS}, 0, rho=g["rho"], lib=lib,
                     device=device, all_nodenames=sputils.create_nodenames_from_branching_factors(BFS))[0]
    oc = oracle_continue_from(ph0, [om.hydro(nm, BFS) for nm in names], g["PHIterLimit"], rho=g["rho"],
                              convthresh=g["convthresh"])
    assert ph._PHIter == oc.iter
    assert rel(conv, oc.conv) < 1e-6
    assert rel(ph.W_array(), oc.W) < 1e-6
    xb = ph.xbar_by_node()
    assert rel(xb["ROOT"][0], oc.xbar[0, :4]) < 1e-8
    for b in range(3):
        assert rel(xb["ROOT_%d" % b][0], oc.xbar[3 * b, 4:]) < 1e-8
        assert rel(xb["ROOT_%d" % b][1], oc.xsqbar[3 * b, 4:]) < 1e-8
    assert rel(ph.nonant_values(), oc.xn()) < 1e-6
    oc.W_on = oc.prox_on = 0
    assert rel(E_nowp, oc.Eobjective()) < 1e-8
    return ph


@pytest.mark.parametrize("native_loop", [1, 0])
def test_hydro_emu(emu, native_loop):
    check_hydro(emu, "cpu", native_loop)


@pytest.mark.gpu
@pytest.mark.parametrize("native_loop", [1, 0])
def test_hydro_gpu(gpu_lib, native_loop):
    ph = check_hydro(gpu_lib, None, native_loop)
    assert hasattr(ph, "iterk_stats") == bool(native_loop)
