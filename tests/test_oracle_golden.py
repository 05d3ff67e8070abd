"""The CPU oracle pinned against the reference's own golden vectors (CPU only).

Each assertion uses a value committed in the reference (tests/golden/ref_goldens.json,
provenance per entry).  The reference's own asserts are loose (places=5 /
1-3 significant digits) because its solvers are ~1e-8..1e-9 accurate; the
oracle (HiGHS + KKT polish) is exact to ~1e-12, so the tolerances below are
the reference's solver noise, not oracle slack.
"""
import json
import os
from math import floor, log10

import numpy as np
import pytest

from oracle import models, ph

def round_pos_sig(x, sig=1):
    """The reference's comparison helper (mpisppy/tests/utils.py:30-31)."""
    return round(x, sig - int(floor(log10(abs(x)))) - 1)


G = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "ref_goldens.json")))


def _farmer3(iters):
    o = ph.OraclePH([models.farmer("scen%d" % i, num_scens=3) for i in range(3)], rho=1.0)
    o.ph_main(iters)
    return o


def test_w_xbar_fixture():
    o = _farmer3(5)
    g = G["farmer3_rho1_5iters"]
    names = ["DevotedAcreage[CORN0]", "DevotedAcreage[SUGAR_BEETS0]", "DevotedAcreage[WHEAT0]"]
    for sn, vn, val in g["W"]:
        k, j = int(sn[4:]), names.index(vn)
        assert o.W[k, j] == pytest.approx(val, abs=10 ** -g["assert_places"])
    for vn, val in g["xbar"]:
        assert o.xbar[0, names.index(vn)] == pytest.approx(val, rel=1e-7)


def test_docs_farmer_trajectory():
    scen = ["good", "average", "bad"]
    o = ph.OraclePH([models.docs_farmer(n) for n in scen], rho=10.0)
    o.ph_main(5, 1e-7)
    for k, n in enumerate(scen):
        ref = G["docs_farmer_rho10_5iters"]["x"][n]
        got = {"X[BEETS]": o.x[k][2], "X[CORN]": o.x[k][1], "X[WHEAT]": o.x[k][0]}
        for vn, val in ref.items():
            assert got[vn] == pytest.approx(val, rel=1e-9)


def test_docs_farmer_ef():
    obj, x, st = ph.solve_ef([models.docs_farmer(n) for n in ["good", "average", "bad"]])
    assert st == "Optimal"
    assert obj == pytest.approx(G["docs_farmer_ef"]["objective"], rel=1e-9)
    assert x[[2, 1, 0]] == pytest.approx([250.0, 80.0, 170.0], rel=1e-9)


def test_farmer30_trivial_bound():
    o = ph.OraclePH([models.farmer("Scenario%d" % i) for i in range(1, 31)], rho=1.0)
    tb = o.iter0()
    ref = G["farmer30_trivial_bound"]["value"]
    assert round_pos_sig(-tb, 3) == round_pos_sig(-ref, 3)      # test_aph.py:246-249
    assert tb == pytest.approx(ref, abs=0.5)


def test_iter0_x_gradient_rho():
    o = ph.OraclePH([models.farmer("scen%d" % i, num_scens=3) for i in range(3)], rho=1.0)
    o.iter0()
    x = o.x[0][o.ncol[0]]
    ref = G["gradient_rho_iter0"]["scen0_x"]
    assert x == pytest.approx([ref["CORN0"], ref["SUGAR_BEETS0"], ref["WHEAT0"]], rel=1e-12)


def test_farmer3_converged_nonants():
    o = ph.OraclePH([models.farmer("scen%d" % i, num_scens=3) for i in range(3)], rho=1.0)
    o.ph_main(500, 1e-4)
    ref = G["farmer3_converged_nonants"]["CORN0,SUGAR_BEETS0,WHEAT0"]
    assert o.xbar[0] == pytest.approx(ref, abs=2e-3)
    assert o.conv < 1e-4


def test_aircond_ef():
    bf = [4, 3, 2]
    obj, x, st = ph.solve_ef([models.aircond("scen%d" % i, bf, start_seed=0) for i in range(24)])
    assert st == "Optimal"
    assert round_pos_sig(obj, 2) == round_pos_sig(G["aircond_ef_bf432"]["objective"], 2)


def test_conv_rank_emulation():
    """convergence_diff = mean over ranks of per-rank means (phbase.py:330-343)."""
    S = 7
    o = ph.OraclePH([models.farmer("scen%d" % i, num_scens=S) for i in range(S)], rho=1.0, n_proc=3)
    o.iter0()
    o.compute_xbar()
    d = np.abs(o.xn() - o.xbar).sum(1)
    sl = ph.rank_slices(S, 3)
    ref = sum(d[s].sum() / (len(s) * o.N) for s in sl) / 3
    assert o.convergence_diff() == pytest.approx(ref, rel=1e-15)


def test_xhat_eval_farmer():
    """Xhat_Eval.evaluate / evaluate_one (test_conf_int_farmer.py:168-202)."""
    g = G["farmer_xhat_eval"]
    scens = [models.farmer("scen%d" % i, num_scens=g["num_scens"]) for i in range(g["names"])]
    E, objs, feas = ph.evaluate_xhat(scens, {"ROOT": g["xhat_ROOT"]})
    assert feas.all()
    assert round_pos_sig(E, g["sig"]) == g["evaluate"]
    assert round_pos_sig(objs[0], g["sig"]) == g["evaluate_one_scen0"]


def test_xhat_eval_aircond():
    """Xhat_Eval.evaluate / evaluate_one, aircond (test_conf_int_aircond.py:213-240)."""
    from mpisppy_amd.utils import sputils
    g = G["aircond_xhat_eval"]
    bf = g["branching_factors"]
    scens = [models.aircond("scen%d" % i, bf, start_seed=0) for i in range(int(np.prod(bf)))]
    cache = {nd: g["xhat_node"] for nd in sputils.create_nodenames_from_branching_factors(bf)}
    E, objs, feas = ph.evaluate_xhat(scens, cache)
    assert feas.all()
    assert round_pos_sig(E, g["sig"]) == g["evaluate"]
    assert round_pos_sig(objs[0], g["sig"]) == g["evaluate_one_scen0"]


def hydro_oracle_ph():
    """Test_hydro.test_ph_solve (test_ef_ph.py:622-640): hydro BF [3,3], rho 1,
    PHIterLimit 10, convthresh 0.001 (test_ef_ph.py:32-52).  The reference's only
    multistage PH pin: conditional prob_coeff (1/9 at ROOT, 1/3 at ROOT_b) and
    per-node x-bar."""
    g = G["hydro_ph_bf33"]
    names = ["Scen%d" % k for k in range(1, 10)]
    o = ph.OraclePH([models.hydro(n, g["branching_factors"]) for n in names], rho=g["rho"])
    conv, Eobj, tb = o.ph_main(g["PHIterLimit"], g["convthresh"])
    o.W_on = o.prox_on = 0                       # ph.disable_W_and_prox()
    return o, conv, Eobj, tb, o.Eobjective()


def test_hydro_ph_pin():
    g = G["hydro_ph_bf33"]
    o, conv, Eobj, tb, E_noWprox = hydro_oracle_ph()
    assert round_pos_sig(tb, g["sig"]) == g["trivial_bound"]
    assert round_pos_sig(E_noWprox, g["sig"]) == g["Eobj_W_prox_disabled"]
    # per-node x-bar: ROOT over all 9 scenarios, each ROOT_b over its 3 (p/uncond = 1/3)
    xn = o.xn()
    o.compute_xbar()
    assert np.allclose(o.xbar[0, :4], xn[:, :4].mean(0), rtol=1e-12, atol=1e-12)
    for b in range(3):
        assert np.allclose(o.xbar[3 * b, 4:], xn[3 * b:3 * b + 3, 4:].mean(0), rtol=1e-12, atol=1e-12)


def test_hydro_ef_pin():
    """Test_hydro.test_ef_solve (test_ef_ph.py:581-601): Scen7.Pgt[2] of the EF ~ 60."""
    g = G["hydro_ph_bf33"]
    scens = [models.hydro("Scen%d" % k, g["branching_factors"]) for k in range(1, 10)]
    obj, x, st = ph.solve_ef(scens)
    n = len(scens[0].c)
    j = scens[6].var_names.index("Pgt[2]")
    assert round_pos_sig(x[6 * n + j], g["ef_sig"]) == g["ef_Scen7_Pgt2"]
