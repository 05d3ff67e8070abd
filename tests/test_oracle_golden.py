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
