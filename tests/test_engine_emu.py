"""The full PH engine (PHBase/PH API) on CPU through the test emulation of the
C ABI (same per-lane solver math as the HIP kernels), against the oracle and
the reference goldens.  The GPU versions of these checks are in test_gpu_parity.py."""
import json
import os

import numpy as np
import pytest

from helpers import all_certified, oracle_continue_from, ph_options, REF_W, REF_XBAR, rel, run_engine
from mpisppy_amd.opt.ph import PH
from mpisppy_amd.examples import aircond, farmer
from mpisppy_amd.utils import sputils
from oracle import models as om, ph as oph

MODES = [{"ipm_after": 0}, {"ipm_after": 256}, {"ipm_after": -1}]


@pytest.fixture(scope="module")
def oracle_farmer30():
    o = oph.OraclePH([om.farmer("scen%d" % i, num_scens=30) for i in range(30)], rho=1.0)
    res = o.ph_main(4)
    return o, res


def test_farmer3_golden_emu(emu):
    ph, conv, Eobj, tb = run_engine(farmer.scenario_creator, farmer.scenario_names_creator(3), {"num_scens": 3},
                                    5, lib=emu, device="cpu")
    assert rel(ph.xbar_by_node()["ROOT"][0], REF_XBAR) < 1e-7
    assert np.max(np.abs(ph.W_array() - REF_W)) < 5e-6


@pytest.mark.parametrize("mode", MODES)
def test_farmer30_modes_vs_oracle(emu, oracle_farmer30, mode):
    o, (oc, oE, otb) = oracle_farmer30
    opts = {"iter0_solver_options": mode, "iterk_solver_options": mode}
    ph, conv, Eobj, tb = run_engine(farmer.scenario_creator, farmer.scenario_names_creator(30), {"num_scens": 30},
                                    4, lib=emu, device="cpu", options=opts)
    assert rel(tb, otb) < 1e-9
    assert rel(ph.xbar_by_node()["ROOT"][0], o.xbar[0]) < 1e-9
    assert rel(ph.W_array(), o.W) < 1e-8
    assert rel(Eobj, oE) < 1e-9
    assert rel(conv, oc) < 1e-8
    assert all(s["not_optimal"] == 0 for s in ph.solve_stats)


def test_per_scenario_models_equal_batch(emu):
    a = run_engine(farmer.scenario_creator, farmer.scenario_names_creator(12), {"num_scens": 12}, 3,
                   lib=emu, device="cpu")
    b = run_engine(farmer.scenario_creator, farmer.scenario_names_creator(12), {"num_scens": 12}, 3,
                   lib=emu, device="cpu", options={"per_scenario_models": True})
    assert np.array_equal(a[0].W_array(), b[0].W_array())
    assert a[1:] == b[1:]


def test_aircond_multistage_emu(emu):
    bfs = [3, 3, 2]
    names = ["scen%d" % i for i in range(18)]
    ph, conv, Eobj, tb = run_engine(aircond.scenario_creator, names, {"branching_factors": bfs, "start_seed": 0},
                                    4, lib=emu, device="cpu",
                                    all_nodenames=sputils.create_nodenames_from_branching_factors(bfs))
    o = oph.OraclePH([om.aircond(n, bfs, start_seed=0) for n in names], rho=1.0)
    oc, oE, otb = o.ph_main(4)
    assert rel(tb, otb) < 1e-12
    assert rel(Eobj, oE) < 1e-10
    assert rel(ph.W_array(), o.W) < 1e-10
    # per-node xbar: 1 ROOT + 3 stage-2 + 9 stage-3 nodes
    xb = ph.xbar_by_node()
    assert len(xb) == 13
    assert rel(xb["ROOT"][0], o.xbar[0, 0:2]) < 1e-12


MULTI_SETTING = (0.2, 4)      # bench.py's C4 solver options (test_bench_settings pins them)


def check_aircond_multi_change(lib, device, bfs, iters, tol_w):
    """The bounded multi-change active-set updates (solver option
    lane_multi_theta, compiled into the lane kernels): the same PH trajectory as
    the oracle's (phbase.py:27-107, 293-343 via oracle/ph.py), and a different
    round path than the single changes (the option is live)."""
    names = ["scen%d" % i for i in range(int(np.prod(bfs)))]
    nodes = sputils.create_nodenames_from_branching_factors(bfs)
    runs = {}
    for th in (0.0, MULTI_SETTING[0]):
        so = {"lane_multi_theta": th, "lane_multi_rounds": MULTI_SETTING[1]}
        runs[th] = run_engine(aircond.scenario_creator, names, {"branching_factors": bfs}, iters, lib=lib,
                              device=device, all_nodenames=nodes,
                              options={"iter0_solver_options": so, "iterk_solver_options": so})
    ph, conv, Eobj, tb = runs[MULTI_SETTING[0]]
    assert all_certified(ph)
    o = oph.OraclePH([om.aircond(n, bfs) for n in names], rho=1.0)
    oc, oE, otb = o.ph_main(iters)
    assert rel(tb, otb) < 1e-9
    assert rel(Eobj, oE) < 1e-8
    assert rel(ph.W_array(), o.W) < tol_w
    assert rel(conv, oc) < 1e-6
    return runs


def test_aircond_multi_change_emu(emu):
    runs = check_aircond_multi_change(emu, "cpu", [10, 10, 3], 3, 1e-8)
    assert not np.array_equal(runs[0.0][0]._host("x"), runs[MULTI_SETTING[0]][0]._host("x"))


@pytest.mark.gpu
def test_aircond_bf10x10x10_multi_change_gpu(gpu_lib):
    """configs[3] with the bench's C4 setting (lane_multi_theta 0.2, 4 rounds)
    through the device loop, vs the oracle (as test_aircond_bf10x10x10_gpu)."""
    runs = check_aircond_multi_change(gpu_lib, None, [10, 10, 10], 3, 1e-6)
    assert hasattr(runs[MULTI_SETTING[0]][0], "iterk_stats")
    assert len(runs[MULTI_SETTING[0]][0].xbar_by_node()) == 111


@pytest.mark.gpu
def test_aircond_all_builds_bit_equal_gpu(gpu_lib, monkeypatch):
    """The small-batch whole-solve kernel's three builds (phx_lane_all: the
    register build; _rl: its data re-loaded per round; _pk: parked in LDS, the
    default where the register build spills) run the same per-lane arithmetic
    on the same values: x, W, x-bar and conv bit for bit equal on configs[3]
    with the bench's C4 setting, and each build is the one that ran."""
    bfs = [10, 10, 10]
    names = ["scen%d" % i for i in range(int(np.prod(bfs)))]
    nodes = sputils.create_nodenames_from_branching_factors(bfs)
    so = {"lane_multi_theta": MULTI_SETTING[0], "lane_multi_rounds": MULTI_SETTING[1]}
    out = {}
    for build, tag in (("reg", ""), ("reload", "all=reload"), ("park", "all=park")):
        monkeypatch.setenv("PHX_ALL_BUILD", build)
        ph, conv, Eobj, tb = run_engine(aircond.scenario_creator, names, {"branching_factors": bfs}, 4,
                                        lib=gpu_lib, all_nodenames=nodes,
                                        options={"iter0_solver_options": so, "iterk_solver_options": so})
        info = ph._native.jit_info(ph._ctx).decode()
        assert (tag in info) if tag else ("all=" not in info), info
        assert all_certified(ph)
        out[build] = (ph._host("x"), ph.W_array(), conv, Eobj)
    for build in ("reload", "park"):
        for a, b in zip(out["reg"], out[build]):
            assert np.array_equal(np.asarray(a), np.asarray(b)), build


def test_docs_farmer_via_engine(emu):
    """doc/src/examples.rst trajectory (rho 10, 5 iterations) through the engine."""
    from mpisppy_amd import model as lm
    from mpisppy_amd.utils import sputils as su

    def build_model(yields):
        m = lm.LinearModel()
        X = m.add_indexed_var("X", ["WHEAT", "CORN", "BEETS"], lb=0.0)
        Y = m.add_indexed_var("Y", ["WHEAT", "CORN"], lb=0.0)
        W = m.add_indexed_var("W", ["WHEAT", "CORN", "BEETS_FAVORABLE", "BEETS_UNFAVORABLE"], lb=0.0)
        plant = 150 * X["WHEAT"] + 230 * X["CORN"] + 260 * X["BEETS"]
        m.set_objective(plant + 238 * Y["WHEAT"] + 210 * Y["CORN"] - 170 * W["WHEAT"] - 150 * W["CORN"]
                        - 36 * W["BEETS_FAVORABLE"] - 10 * W["BEETS_UNFAVORABLE"])
        m.add_constraint(X["WHEAT"] + X["CORN"] + X["BEETS"], ub=500)
        m.add_constraint(yields[0] * X["WHEAT"] + Y["WHEAT"] - W["WHEAT"], lb=200)
        m.add_constraint(yields[1] * X["CORN"] + Y["CORN"] - W["CORN"], lb=240)
        m.add_constraint(yields[2] * X["BEETS"] - W["BEETS_FAVORABLE"] - W["BEETS_UNFAVORABLE"], lb=0)
        W["BEETS_FAVORABLE"].ub = 6000
        return m, plant, X

    def scenario_creator(name):
        y = {"good": [3, 3.6, 24], "average": [2.5, 3, 20], "bad": [2, 2.4, 16]}[name]
        m, plant, X = build_model(y)
        su.attach_root_node(m, plant, [X])
        m._mpisppy_probability = 1.0 / 3
        return m

    ph, conv, Eobj, tb = run_engine(scenario_creator, ["good", "average", "bad"], None, 5, rho=10.0,
                                    lib=emu, device="cpu")
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "ref_goldens.json")))
    vals = ph.gather_var_values_to_rank0()
    for sn, ref in g["docs_farmer_rho10_5iters"]["x"].items():
        for vn, v in ref.items():
            assert vals[sn, vn] == pytest.approx(v, rel=1e-9)


def test_maximize_sense(emu):
    """max problems: PH term subtracted (phbase.py:696-699); same x, negated objective."""
    from mpisppy_amd import model as lm
    a = run_engine(farmer.scenario_creator, farmer.scenario_names_creator(6), {"num_scens": 6}, 3,
                   lib=emu, device="cpu")
    b = run_engine(farmer.scenario_creator, farmer.scenario_names_creator(6),
                   {"num_scens": 6, "sense": lm.maximize}, 3, lib=emu, device="cpu")
    assert rel(a[0].W_array(), -b[0].W_array()) < 1e-9 or rel(a[0].nonant_values(), b[0].nonant_values()) < 1e-9
    assert rel(a[3], -b[3]) < 1e-12           # trivial bound
    assert rel(a[2], -b[2]) < 1e-9            # Eobj
    assert rel(a[0].nonant_values(), b[0].nonant_values()) < 1e-9


def test_conv_emulated_ranks(emu):
    """options['conv_ranks'] reproduces the reference's per-rank-mean conv for R ranks."""
    S = 10
    o = oph.OraclePH([om.farmer("scen%d" % i, num_scens=S) for i in range(S)], rho=1.0, n_proc=3)
    oc, oE, otb = o.ph_main(2)
    ph, conv, Eobj, tb = run_engine(farmer.scenario_creator, farmer.scenario_names_creator(S), {"num_scens": S},
                                    2, lib=emu, device="cpu", options={"conv_ranks": 3})
    assert rel(conv, oc) < 1e-9


def test_convthresh_stops_before_solve(emu):
    """Stop test is strict and happens before the iteration's solve (phbase.py:930-934)."""
    ph, conv, Eobj, tb = run_engine(farmer.scenario_creator, farmer.scenario_names_creator(3), {"num_scens": 3},
                                    500, lib=emu, device="cpu", options={"convthresh": 1e-4})
    o = oph.OraclePH([om.farmer("scen%d" % i, num_scens=3) for i in range(3)], rho=1.0)
    it = o.iterk(500, 1e-4) if o.iter0() is not None else None
    assert ph._PHIter == it
    assert conv < 1e-4


@pytest.mark.parametrize("so", [{"as_rounds": 0, "ipm_max_it": 2}, {"as_rounds": 1, "ipm_max_it": 3}])
def test_deferred_solve_with_stragglers_matches_sync(emu, so):
    """Deferred solves (phx_solve opts.defer) let Compute_Xbar/Update_W run
    behind the solve; when scenarios must go to the generic path (forced here by
    starving the interior point), convergence_diff finishes the solve and redoes
    the step.  The trajectory must equal the synchronous one."""
    S = 24
    runs = []
    for defer in (1, 0):
        o = dict(so, defer=defer, native_loop=0)
        ph, conv, Eobj, tb = run_engine(farmer.scenario_creator, farmer.scenario_names_creator(S),
                                        {"num_scens": S}, 4, lib=emu, device="cpu",
                                        options={"iter0_solver_options": o, "iterk_solver_options": o})
        runs.append((ph, conv, Eobj, tb))
    (a, ca, Ea, ta), (b, cb, Eb, tb_) = runs
    assert any(s.get("stragglers", 0) > 0 for s in a.solve_stats)
    assert np.array_equal(a.W_array(), b.W_array())
    assert np.array_equal(a.xbar_by_node()["ROOT"][0], b.xbar_by_node()["ROOT"][0])
    assert ca == cb and Ea == Eb and ta == tb_


@pytest.mark.parametrize("case", ["farmer", "aircond", "conv_ranks", "converge"])
def test_native_loop_matches_host_loop_emu(emu, case):
    """phx_iterk (device-driven iterk_loop) against the Python loop of PHBase
    methods: the same iterations, bit for bit."""
    check_native_vs_host(emu, "cpu", case)


def check_native_vs_host(lib, device, case, S=30, solver=None, fused=0):
    """fused=0: bit for bit.  fused=1 (GPU): phx_iterk's one-launch-per-iteration
    mode sums x-bar and conv in another fixed order, so they agree to 1e-9."""
    runs = []
    for nl in (1, 0):
        so = dict(solver or {}, native_loop=nl)
        if nl:
            so["iterk_fused"] = fused
        opts = {"iter0_solver_options": dict(solver or {}), "iterk_solver_options": so}
        kw = dict(lib=lib, device=device, options=opts)
        if case == "aircond":
            bfs = [3, 3, 2]
            r = run_engine(aircond.scenario_creator, ["scen%d" % i for i in range(18)],
                           {"branching_factors": bfs, "start_seed": 0}, 5,
                           all_nodenames=sputils.create_nodenames_from_branching_factors(bfs), **kw)
        else:
            iters = 400 if case == "converge" else 5
            if case == "conv_ranks":
                opts["conv_ranks"] = 4
            if case == "converge":
                opts["convthresh"] = 1e-3
                S = 30                   # converges within the 400 iterations
            r = run_engine(farmer.scenario_creator, farmer.scenario_names_creator(S), {"num_scens": S}, iters,
                           **kw)
        runs.append(r)
    (a, ca, Ea, ta), (b, cb, Eb, tb_) = runs
    assert hasattr(a, "iterk_stats") and not hasattr(b, "iterk_stats")
    assert a._PHIter == b._PHIter
    if case == "converge":
        assert a.iterk_stats["converged"] and a._PHIter < 400
    if fused:
        assert a.iterk_stats["fused"] == (case in ("farmer", "converge"))
        if a.iterk_stats["fused"]:
            def rel(u, v):
                u, v = np.asarray(u, dtype=float), np.asarray(v, dtype=float)
                return float(np.max(np.abs(u - v) / np.maximum(1.0, np.abs(v)))) if u.size else 0.0
            assert rel(a.W_array(), b.W_array()) < 1e-9
            assert rel(a.nonant_values(), b.nonant_values()) < 1e-9
            for k, v in b.xbar_by_node().items():
                assert rel(a.xbar_by_node()[k][0], v[0]) < 1e-9
            assert rel(ca, cb) < 1e-9 and rel(Ea, Eb) < 1e-9 and ta == tb_
            return a, b
    assert not a.iterk_stats.get("fused", False)
    assert np.array_equal(a.W_array(), b.W_array())
    assert np.array_equal(a.nonant_values(), b.nonant_values())
    for k, v in b.xbar_by_node().items():
        assert np.array_equal(a.xbar_by_node()[k][0], v[0])
    assert ca == cb and Ea == Eb and ta == tb_
    return a, b


def test_farmer_cm10_workgroup_warm_pass(emu):
    """farmer crops_multiplier=10 (n=120, above the lane limits: generic path).
    The workgroup warm active-set pass (phx_wg.h) must certify the later PH
    iterations without PDHG and give the same PH trajectory as the PDHG + polish
    path and the oracle (ph loop pinned by test_oracle_golden.py)."""
    S, it = 6, 4
    kw = {"num_scens": S, "crops_multiplier": 10}
    res = {}
    for wg in (1, 0):
        so = {"wg_warm": 16 * wg, "native_loop": 0}   # per-solve statistics: the host loop
        res[wg] = run_engine(farmer.scenario_creator, farmer.scenario_names_creator(S), kw, it, lib=emu,
                             device="cpu", options={"iter0_solver_options": so, "iterk_solver_options": so})
    ph1, ph0 = res[1][0], res[0][0]
    wgc = [r["wg_certified"] for r in ph1.solve_stats]
    assert wgc[0] == 0 and wgc[-1] == S and wgc[-2] == S, wgc
    assert all(r["pdhg_iters"] == 0 for r in ph1.solve_stats[-2:])
    assert all(r["wg_certified"] == 0 for r in ph0.solve_stats)
    assert all(r["not_optimal"] == 0 for r in ph1.solve_stats)
    assert rel(ph1.xbar_by_node()["ROOT"][0], ph0.xbar_by_node()["ROOT"][0]) < 1e-9
    assert rel(ph1.W_array(), ph0.W_array()) < 1e-8
    # Iter0 LPs are degenerate at crops_multiplier=10 (equal optimum, different
    # vertices), so check as test_sslp does: trivial bound, then the last
    # iteration's subproblems re-solved by the oracle from the engine's own W /
    # x-bar (unique nonant optimum under the prox term)
    o = oph.OraclePH([om.farmer("scen%d" % i, crops_multiplier=10, num_scens=S) for i in range(S)], rho=1.0)
    assert rel(res[1][3], o.iter0()) < 1e-9
    o.W = ph1.W_array().copy()
    o.xbar = np.tile(ph1.xbar_by_node()["ROOT"][0], (S, 1))
    o.W_on, o.prox_on = 1, 1
    o.solve_loop()
    # the oracle's point is KKT-certified (oracle/qp.py certified_polish), so the
    # unique nonant optimum under the prox term is the bar (north_star: 1e-6)
    assert rel(ph1._host("obj"), o.obj) < 1e-8
    assert rel(ph1.nonant_values(), o.xn()) < 1e-6
    # full W / x-bar trajectory: the oracle's iterations 1..it from the engine's Iter0 point
    ph00 = run_engine(farmer.scenario_creator, farmer.scenario_names_creator(S), kw, 0, lib=emu, device="cpu")[0]
    oc = oracle_continue_from(ph00, [om.farmer("scen%d" % i, crops_multiplier=10, num_scens=S) for i in range(S)], it)
    assert rel(ph1.W_array(), oc.W) < 1e-6
    assert rel(ph1.xbar_by_node()["ROOT"][0], oc.xbar[0]) < 1e-8


def test_time_to_conv_emu(emu):
    """farmer-3 to conv < 1e-4 through the emulated phx_iterk: the oracle's stop
    iteration (94) and the reference's converged nonants (test_gpu_parity.py)."""
    import test_gpu_parity as tg
    ph = tg.check_time_to_conv(emu, "cpu", 3)
    assert ph._PHIter == 94


def check_native_vs_host_wg(lib, device, S=20, iters=5, solver=None, iterk_extra=None):
    """Subproblems above the lane solver's limits (farmer crops_multiplier=10):
    phx_iterk runs the workgroup warm pass per iteration (stragglers through
    the stop / finish / resume protocol) == the host loop, bit for bit.
    iterk_extra: solver options of the PH iterations only."""
    runs = []
    for nl in (1, 0):
        so = dict(solver or {}, native_loop=nl, **(iterk_extra or {}))
        opts = {"iter0_solver_options": dict(solver or {}), "iterk_solver_options": so}
        runs.append(run_engine(farmer.scenario_creator, farmer.scenario_names_creator(S),
                               {"num_scens": S, "crops_multiplier": 10}, iters, lib=lib, device=device,
                               options=opts))
    (a, ca, Ea, ta), (b, cb, Eb, tb_) = runs
    assert hasattr(a, "iterk_stats") and not hasattr(b, "iterk_stats")
    assert not a._native.jit_info(a._ctx).decode().startswith("on")
    assert a._PHIter == b._PHIter
    assert np.array_equal(a.W_array(), b.W_array())
    assert np.array_equal(a.nonant_values(), b.nonant_values())
    assert ca == cb and Ea == Eb and ta == tb_
    return a, b


def test_native_loop_workgroup_matches_host_loop_emu(emu):
    check_native_vs_host_wg(emu, "cpu")


def test_native_loop_workgroup_stragglers_emu(emu):
    """One workgroup round per solve: lanes left to PDHG + polish stop the
    device loop, which finishes them and resumes (same trajectory)."""
    check_native_vs_host_wg(emu, "cpu", solver={"wg_warm": 1})   # (the stop count: GPU test)


def check_reductions_by_iteration(lib, device, S, fused, K=3, rho=1.0):
    """Compute_Xbar / Update_W / convergence_diff at full size, recomputed on the host
    from the engine's own x (phbase.py:27-107, 293-343): runs with PHIterLimit =
    0..K are deterministic prefixes of one another, so run k-1's nonants and W are
    the inputs of run k's last iteration; its x-bar / x-sq-bar (math.fsum of
    prob_coeff * x), W = W_old + rho (x - x-bar) and conv must agree to 1e-12
    relative.  At S = 100,000 this checks the multi-tile / sharded-arrival reductions
    (k_xbar, k_update_w_seg; in fused mode the warm kernel's x-bar partials from
    iteration 2 on) independently of the oracle."""
    import math
    so = {"iterk_fused": fused}
    runs = []
    for k in range(K + 1):
        ph, conv, Eobj, tb = run_engine(farmer.scenario_creator, farmer.scenario_names_creator(S),
                                        {"num_scens": S}, k, rho=rho, lib=lib, device=device,
                                        options={"iter0_solver_options": so, "iterk_solver_options": so})
        assert all_certified(ph)
        xb, xsq = ph.xbar_by_node()["ROOT"]
        runs.append(dict(xn=ph.nonant_values(), W=ph.W_array(), xb=xb, xsq=xsq, conv=ph.conv,
                         pc=ph._prob_coeff.copy(), fused=getattr(ph, "iterk_stats", {}).get("fused")))
        del ph
    for k in range(1, K + 1):
        prev, cur = runs[k - 1], runs[k]
        x, pc = prev["xn"], cur["pc"]
        N = x.shape[1]
        xb = np.array([math.fsum(pc[j] * x[:, j]) for j in range(N)])
        xsq = np.array([math.fsum(pc[j] * x[:, j] * x[:, j]) for j in range(N)])
        W = prev["W"] + rho * (x - xb[None, :])
        conv = math.fsum(np.abs(x - xb[None, :]).ravel()) / (S * N)
        assert rel(cur["xb"], xb) < 1e-12, k
        assert rel(cur["xsq"], xsq) < 1e-12, k
        assert rel(cur["W"], W) < 1e-12, k
        assert abs(cur["conv"] - conv) <= 1e-12 * max(1.0, conv), k
    return runs


@pytest.mark.parametrize("fused", [0, 1])
def test_reductions_by_iteration_emu(emu, fused):
    check_reductions_by_iteration(emu, "cpu", 3000, fused)


def check_wg_factor_cache(lib, device, monkeypatch, S=60, iters=6):
    """The workgroup warm solver's factor cache (phx_wg.h WgPairs::fac: the
    factor of the last active set reused while the set and the prox weights are
    unchanged) gives the PH trajectory of recomputing every factor, bit for bit
    (farmer crops_multiplier=10: n = 120, above the lane solver's limits)."""
    kw = {"num_scens": S, "crops_multiplier": 10}
    out = []
    for off in (False, True):
        if off:
            monkeypatch.setenv("PHX_WG_NO_FACTOR_CACHE", "1")
        ph, conv, Eobj, tb = run_engine(farmer.scenario_creator, farmer.scenario_names_creator(S), kw, iters,
                                        lib=lib, device=device)
        assert all_certified(ph)
        assert ("factor cache" in ph._native.jit_info(ph._ctx).decode()) != off
        out.append((ph.W_array(), ph.xbar_by_node()["ROOT"][0], conv, Eobj))
    monkeypatch.delenv("PHX_WG_NO_FACTOR_CACHE")
    (W0, x0, c0, E0), (W1, x1, c1, E1) = out
    assert np.array_equal(W0, W1) and np.array_equal(x0, x1) and c0 == c1 and E0 == E1


def test_wg_factor_cache_emu(emu, monkeypatch):
    check_wg_factor_cache(emu, "cpu", monkeypatch)


def check_deferred_iter0(lib, device, S=600, iter0_solver=None, iters=5):
    """PH.ph_main defers Iter0's host synchronisation: its E1 / feasibility checks
    and trivial bound run after the device loop, which adopts Iter0's pending
    solve (phx_iterk; lanes that solve leaves to the generic path stop the
    pipeline at iteration 1, are finished, and the loop resumes).  The result is
    the step-by-step run's (Iter0() then iterk_loop()), bit for bit."""
    from mpisppy_amd.opt.ph import PH
    from helpers import ph_options

    def make():
        opts = ph_options(iters)
        opts["iter0_solver_options"] = dict(iter0_solver or {})
        return PH(opts, farmer.scenario_names_creator(S), farmer.scenario_creator,
                  scenario_creator_kwargs={"num_scens": S}, _native_lib=lib, _device=device)
    a = make()
    ca, Ea, ta = a.ph_main()
    assert getattr(a, "_iter0_was_deferred", False)
    b = make()
    b.PH_Prep()
    b.subproblem_creation(False)
    tb = b.Iter0()
    assert not getattr(b, "_iter0_deferred", False) and tb is not None
    b.iterk_loop()
    Eb = b.post_loops()
    assert ta == tb and ca == b.conv and Ea == Eb
    assert np.array_equal(a.W_array(), b.W_array())
    assert np.array_equal(a.xbar_by_node()["ROOT"][0], b.xbar_by_node()["ROOT"][0])
    assert a.E1 == b.E1 == pytest.approx(1.0)
    assert np.array_equal(a._iter0_obj, b._iter0_obj)
    return a, b


@pytest.mark.parametrize("so0", [None, {"as_rounds": 0, "ipm_max_it": 2}])
def test_deferred_iter0_emu(emu, so0):
    a, b = check_deferred_iter0(emu, "cpu", iter0_solver=so0)
    if so0:
        assert a.solve_stats[0]["stragglers"] > 0      # Iter0's leftovers finished after adoption


def infeasible_farmer_creator(sname, **kw):
    """farmer, except scen1 must plant 400 + 400 acres of wheat and corn on a
    500-acre farm: its Iter0 LP is infeasible."""
    m = farmer.scenario_creator(sname, **kw)
    if sname == "scen1":
        m.DevotedAcreage["WHEAT0"].lb = 400.0
        m.DevotedAcreage["CORN0"].lb = 400.0
    return m


def check_infeasible_deferred_iter0(lib, device, S=30):
    """ph_main defers Iter0's checks to the device loop; an Iter0 with an
    infeasible scenario still quits before any PH iteration runs, as the
    reference does right after Iter0 (phbase.py:812-823): phx_iterk stops
    after adopting that solve (no iteration ran) and the checks quit()."""
    ph = PH(ph_options(20), farmer.scenario_names_creator(S), infeasible_farmer_creator,
            scenario_creator_kwargs={"num_scens": S}, _native_lib=lib, _device=device)
    seen = []
    orig = ph._native.iterk

    def spy(ctx, so, a, res, stream):
        rc = orig(ctx, so, a, res, stream)
        seen.append((res._obj.iters, res._obj.solves, res._obj.adopted))
        return rc
    ph._native.iterk = spy
    with pytest.raises(SystemExit):
        ph.ph_main()
    ph._native.iterk = orig
    assert seen == [(0, 0, 1)], seen          # adopted Iter0, no PH iteration
    assert ph.E1 == pytest.approx(1.0)


def test_infeasible_deferred_iter0_emu(emu):
    check_infeasible_deferred_iter0(emu, "cpu")


def check_infeasible_iter0_status(lib, device, S=30):
    """The infeasible scenario is never certified (its lane-solver refinement
    diverges to a non-finite point, which every KKT certificate must reject --
    before round 4 a NaN point passed them all and was reported OPTIMAL): it
    ends without an optimal status (here the generic path's iteration limit:
    its interior point finds no Farkas certificate with margin for this
    instance) while every other scenario is optimal and finite, and Iter0's
    feasibility check quits (phbase.py:818-823)."""
    ph = PH(ph_options(0), farmer.scenario_names_creator(S), infeasible_farmer_creator,
            scenario_creator_kwargs={"num_scens": S}, _native_lib=lib, _device=device)
    ph.PH_Prep()
    ph.subproblem_creation(False)
    with pytest.raises(SystemExit):
        ph.Iter0()
    st = ph._status.cpu().numpy()
    assert st[1] != 1, st[:4]
    assert (np.delete(st, 1) == 1).all()
    x = ph._host("x")
    assert np.isfinite(np.delete(x, 1, axis=1)).all()
    assert ph.solve_stats[-1]["not_optimal"] == 1


def test_infeasible_iter0_status_emu(emu):
    check_infeasible_iter0_status(emu, "cpu")
