"""netdes LP relaxation (workload C5b): the restated scenario creator
(batch == per-scenario models, bit-exact; == the oracle's dense restatement), and PH
through the engine against the oracle on the shipped network-10-10-H-01 instance
(n = 108, m = 64, 54 nonants, scenario-varying A, c and right-hand sides, shipped
non-uniform probabilities).  The reference ships no netdes LP-relaxation golden values
(solutions.dat holds MIP optima; asserted here only as an upper bound on the LP
trivial bound): parity is engine vs the oracle restatement, whose PH loop is pinned by
the farmer/aircond goldens (test_oracle_golden.py)."""
import numpy as np
import pytest

from helpers import all_certified, rel, run_engine
from mpisppy_amd.batch import from_models
from mpisppy_amd.examples import netdes
from oracle import models as om, ph as oph

INST = "network-10-10-H-01"
MIP_OPT = 27523.7          # examples/netdes/solutions.dat, network-10-10-H-01 best bound


def test_netdes_batch_equals_models():
    names = netdes.scenario_names_creator(10)       # the shipped scenarios, shipped probabilities
    a = from_models(names, [netdes.scenario_creator(nm, path="data/%s.dat" % INST) for nm in names]).compress()
    b = netdes.batch_creator(names, instance=INST).compress()
    for k in ["rowptr", "colidx", "kvar", "Aconst", "Avar", "c", "lb", "ub", "bl", "bu"]:
        assert np.array_equal(getattr(a, k), getattr(b, k)), k
    assert (a.n, a.m) == (108, 64) and a.nnz == b.nnz == 2 * 54 + 2 * 54
    assert list(a.nonant.slot_col) == list(range(54)) and a.rhs_vary and a.c_vary
    assert a.prob == b.prob and abs(sum(a.prob) - 1.0) < 1e-12
    names = netdes.scenario_names_creator(12)       # 10..11 synthetic: only with num_scens
    a = from_models(names, [netdes.scenario_creator(nm, instance=INST, num_scens=12) for nm in names]).compress()
    b = netdes.batch_creator(names, instance=INST, num_scens=12).compress()
    for k in ["Avar", "c", "bl", "bu"]:
        assert np.array_equal(getattr(a, k), getattr(b, k)), k
    assert a.prob == b.prob == [1 / 12] * 12
    with pytest.raises(ValueError):                 # parse.py:34-37
        netdes.scenario_creator("Scenario10", instance=INST)
    with pytest.raises(ValueError):
        netdes.batch_creator(names, instance=INST)
    with pytest.raises(RuntimeError):
        netdes.scenario_creator("Scenario0")
    assert netdes._get_scenario_ix("Scen07") == 7


def test_netdes_oracle_model_matches_creator():
    for nm, ns in [("Scenario3", None), ("Scenario17", 20)]:
        sf = netdes.scenario_creator(nm, instance=INST, num_scens=ns).standard_form()
        o = om.netdes(nm, INST, num_scens=ns)
        A = np.zeros((len(sf["bl"]), len(sf["c"])))
        for i in range(len(sf["bl"])):
            for k in range(sf["rowptr"][i], sf["rowptr"][i + 1]):
                A[i, sf["colidx"][k]] = sf["vals"][k]
        assert np.array_equal(A, o.A) and np.array_equal(sf["c"], o.c)
        assert np.array_equal(sf["bl"], o.bl) and np.array_equal(sf["bu"], o.bu)
        assert np.array_equal(sf["lb"], o.lb) and np.array_equal(sf["ub"], o.ub)


def test_netdes_oracle_trivial_bound_below_mip():
    o = oph.OraclePH([om.netdes(nm, INST) for nm in netdes.scenario_names_creator(10)], rho=1.0)
    tb = o.iter0()
    assert 0.0 < tb <= MIP_OPT


def check_netdes_ph(lib, device, iters=3):
    """Iter0 LPs may be degenerate, so engine and oracle trajectories can differ;
    checked: the trivial bound (unique LP optimum value) to 1e-8, and every subproblem
    of the last iteration re-solved by the oracle from the engine's own W / x-bar: the
    nonants to 1e-6 and the objectives to 1e-8 (north_star bar)."""
    names = netdes.scenario_names_creator(10)
    ph, conv, Eobj, tb = run_engine(netdes.scenario_creator, names, {"instance": INST}, iters, lib=lib,
                                    device=device, options={"per_scenario_models": True})
    o = oph.OraclePH([om.netdes(nm, INST) for nm in names], rho=1.0)
    otb = o.iter0()
    assert rel(tb, otb) < 1e-8
    assert all_certified(ph)
    o.W = ph.W_array().copy()
    o.xbar = np.tile(ph.xbar_by_node()["ROOT"][0], (len(names), 1))
    o.W_on, o.prox_on = 1, 1
    o.solve_loop()
    assert rel(ph.nonant_values(), o.xn()) < 1e-6
    assert rel(ph._host("obj"), o.obj) < 1e-8
    return ph, o


def test_netdes_ph_emu(emu):
    check_netdes_ph(emu, "cpu", iters=2)


@pytest.mark.gpu
def test_netdes_ph_gpu(gpu_lib):
    check_netdes_ph(gpu_lib, None, iters=3)


@pytest.mark.gpu
def test_netdes_synthetic_batch_gpu(gpu_lib):
    """200 scenarios (10 shipped + 190 synthetic, batch creator, p = 1/200): every
    subproblem certified; the last iteration re-solved by the oracle from the engine's
    W / x-bar agrees to 1e-6 on a sample of scenarios."""
    names = netdes.scenario_names_creator(200)
    ph, conv, Eobj, tb = run_engine(netdes.scenario_creator, names, {"instance": INST, "num_scens": 200}, 3,
                                    lib=gpu_lib)
    assert all_certified(ph)
    pick = [0, 7, 10, 99, 199]
    o = oph.OraclePH([om.netdes(names[k], INST, num_scens=200) for k in pick], rho=1.0)
    o.iter0()
    o.W = ph.W_array()[pick].copy()
    o.xbar = np.tile(ph.xbar_by_node()["ROOT"][0], (len(pick), 1))
    o.W_on, o.prox_on = 1, 1
    o.solve_loop()
    assert rel(ph.nonant_values()[pick], o.xn()) < 1e-6


# ---- C5b: network-50-30-H (n = 2,940, m = 1,520, 1,470 nonants) through the sparse
#      workgroup solver (phx_sp.h) -------------------------------------------------
INST50 = "network-50-30-H-01"
HIGHS_LP_50 = 75593.51224584531   # round-1 HiGHS LP value of the 30 shipped scenarios


def check_netdes50(lib, device, S, iters, pick, solver=None):
    """S scenarios of network-50-30-H (the 30 shipped ones when S == 30, else the
    synthetic workload: shipped k mod 30 with perturbed costs, p = 1/S), `iters` PH
    iterations.  Every subproblem of every solve is certified; the trivial bound
    matches the oracle's (HiGHS LP + certified polish) on the sampled scenarios'
    LPs; the last iteration's subproblems of the sample, re-solved by the oracle
    (independent sparse interior point + certified active-set polish) from the
    engine's own W / x-bar, agree to 1e-6 in the nonants and 1e-8 in objective."""
    names = netdes.scenario_names_creator(S)
    kw = {"instance": INST50}
    okw = {}
    if S != 30:
        kw["num_scens"] = okw["num_scens"] = S
    opts = {}
    if solver:
        opts = {"iter0_solver_options": dict(solver), "iterk_solver_options": dict(solver)}
    ph, conv, Eobj, tb = run_engine(netdes.scenario_creator, names, kw, iters, lib=lib, device=device,
                                    options=opts)
    assert all_certified(ph), [s["not_optimal"] for s in ph.solve_stats]
    o = oph.OraclePH([om.netdes(names[k], INST50, **okw) for k in pick], rho=1.0)
    o.iter0()
    # Iter0 objective per sampled scenario (unique LP optimum value)
    assert rel(ph._iter0_obj[pick], o.obj) < 1e-8
    if S == 30:
        assert rel(tb, HIGHS_LP_50) < 1e-9
    o.W = ph.W_array()[pick].copy()
    o.xbar = np.tile(ph.xbar_by_node()["ROOT"][0], (len(pick), 1))
    o.W_on, o.prox_on = 1, 1
    o.solve_loop()
    assert rel(ph.nonant_values()[pick], o.xn()) < 1e-6
    assert rel(ph._host("obj")[pick], o.obj) < 1e-8
    return ph


def test_netdes50_sparse_emu(emu):
    ph = check_netdes50(emu, "cpu", 30, 3, [0, 7, 19, 29])
    st = ph.solve_stats
    assert st[0]["sp_certified"] == 30 and st[0]["sp_ipm_its"] > 0
    assert all(s["sp_certified"] == 30 and s["sp_ipm_its"] == 0 for s in st[1:])   # warm rounds only


def test_sparse_alone_and_dense_paths_emu(emu, monkeypatch):
    """netdes-10 (n = 108: beyond the lane solver) through the sparse solver alone
    (PHX_NO_WG=1: no dense workgroup warm pass) and through the dense generic path
    (PHX_SP=0: PDHG + dense polish / IPM, the round-1 path): both match the oracle."""
    monkeypatch.setenv("PHX_NO_WG", "1")
    ph, o = check_netdes_ph(emu, "cpu", iters=3)
    assert all(s["sp_certified"] == 10 for s in ph.solve_stats)
    monkeypatch.delenv("PHX_NO_WG")
    monkeypatch.setenv("PHX_SP", "0")
    ph, o = check_netdes_ph(emu, "cpu", iters=2)
    assert all(s["sp_certified"] == 0 for s in ph.solve_stats)


@pytest.mark.gpu
def test_netdes50_shipped_gpu(gpu_lib):
    check_netdes50(gpu_lib, None, 30, 4, list(range(30)))


@pytest.mark.gpu
def test_netdes50_10k_gpu(gpu_lib):
    """BASELINE configs[4], C5b at full size: 10,000 scenarios, 3 PH iterations."""
    ph = check_netdes50(gpu_lib, None, 10000, 3, [0, 1, 29, 30, 4999, 9998, 9999])
    print({k: [s[k] for s in ph.solve_stats] for k in ["sp_certified", "sp_ms", "sp_ipm_its", "sp_warm_rounds",
                                                       "pdhg_iters", "wall_s"]})


def check_native_vs_host_sp(lib, device, inst, S, iters):
    """Subproblems above the workgroup limits: phx_iterk runs the sparse solver's
    warm pass per iteration (k_sp_solve, stragglers through the stop / finish /
    resume protocol) == the host loop (phx_solve -> finish_run), bit for bit."""
    names = netdes.scenario_names_creator(S)
    runs = []
    for nl in (1, 0):
        opts = {"iterk_solver_options": {"native_loop": nl}}
        runs.append(run_engine(netdes.scenario_creator, names, {"instance": inst}, iters, lib=lib, device=device,
                               options=opts))
    (a, ca, Ea, ta), (b, cb, Eb, tb_) = runs
    assert hasattr(a, "iterk_stats") and not hasattr(b, "iterk_stats")
    info = a._native.jit_info(a._ctx).decode()
    assert "sparse solver on" in info and "workgroup solver on" not in info, info
    assert a._PHIter == b._PHIter == iters
    assert np.array_equal(a.W_array(), b.W_array())
    assert np.array_equal(a.nonant_values(), b.nonant_values())
    assert ca == cb and Ea == Eb and ta == tb_
    assert all_certified(a) and all_certified(b)
    return a, b


def test_native_loop_sparse_matches_host_loop_emu(emu, monkeypatch):
    monkeypatch.setenv("PHX_NO_WG", "1")             # netdes-10 would fit the workgroup solver
    check_native_vs_host_sp(emu, "cpu", INST, 10, 3)


@pytest.mark.gpu
def test_native_loop_sparse_matches_host_loop_gpu(gpu_lib):
    """C5b's loop (network-50-30-H, the 30 shipped scenarios) through phx_iterk."""
    a, b = check_native_vs_host_sp(gpu_lib, None, INST50, 30, 4)
    assert a.iterk_stats["iters"] == 4
