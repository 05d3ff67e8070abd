"""variable_probability (spbase.py:394-452, phbase.py:27-107 and 314-318): per
(scenario, nonant) probabilities replace prob_coeff in x-bar, zero-probability
nonants keep W = 0, and the sums per node and variable must be one.  Checked
against the oracle with the same per-slot probabilities (CPU, emulation)."""
import numpy as np
import pytest

from helpers import ph_options, rel
from mpisppy_amd.examples import farmer
from mpisppy_amd.opt.ph import PH
from oracle import models as om, ph as oph

S = 3
CROPS = ["WHEAT0", "CORN0", "SUGAR_BEETS0"]
# per scenario, per crop: the wheat acreage is decided by scenarios 0 and 1 only
PROBS = {0: [0.5, 1 / 3, 1 / 3], 1: [0.5, 1 / 3, 1 / 3], 2: [0.0, 1 / 3, 1 / 3]}


def _vp(model):
    return [(id(model.DevotedAcreage[c]), PROBS[_num(model)][i]) for i, c in enumerate(CROPS)]


def _num(model):
    names = {"BelowAverageScenario0": 0, "AverageScenario0": 1, "AboveAverageScenario0": 2}
    return names[model.name]


def _run(lib, vp, iters=5):
    ph = PH(ph_options(iters), farmer.scenario_names_creator(S), farmer.scenario_creator,
            scenario_creator_kwargs={"num_scens": S}, variable_probability=vp, _native_lib=lib, _device="cpu")
    conv, Eobj, tb = ph.ph_main()
    return ph, conv, Eobj, tb


def test_default_probabilities_change_nothing(emu):
    def vp(model):
        return [(id(model.DevotedAcreage[c]), 1.0 / S) for c in CROPS]
    a = _run(emu, vp)
    b = _run(emu, None)
    assert np.array_equal(a[0].W_array(), b[0].W_array())
    assert a[1] == b[1] and a[2] == b[2] and a[3] == b[3]


def test_variable_probability_matches_oracle(emu):
    ph, conv, Eobj, tb = _run(emu, _vp, iters=6)
    o = oph.OraclePH([om.farmer("scen%d" % i, num_scens=S) for i in range(S)], rho=1.0)
    # the same probabilities in slot order (nonant slots are sorted by name)
    order = [CROPS.index(nm.split("[")[1].rstrip("]")) for nm in ph.batch.nonant.var_names]
    P = np.array([[PROBS[k][c] for c in order] for k in range(S)])
    o.pc[:] = P
    o.prob0_mask = (P != 0).astype(float)
    oc, oE, otb = o.ph_main(6)
    assert rel(ph.W_array(), o.W) < 1e-7
    assert np.all(ph.W_array()[P == 0] == 0.0)        # zero probability: W stays 0
    assert rel(ph.xbar_by_node()["ROOT"][0], o.xbar[0]) < 1e-7
    assert rel(conv, oc) < 1e-7 and rel(Eobj, oE) < 1e-9 and rel(tb, otb) < 1e-9
    assert not hasattr(ph, "iterk_stats")             # the W mask runs in the host loop
    m2 = ph._models["scen2"]
    assert ph.is_zero_prob(m2, m2.DevotedAcreage["WHEAT0"])
    assert not ph.is_zero_prob(m2, m2.DevotedAcreage["CORN0"])


def test_probability_sums_checked(emu):
    def bad(model):
        return [(id(model.DevotedAcreage["WHEAT0"]), 0.5)]
    with pytest.raises(RuntimeError, match="not 1"):
        _run(emu, bad)
    opts = ph_options(2)
    opts["do_not_check_variable_probabilities"] = True
    PH(opts, farmer.scenario_names_creator(S), farmer.scenario_creator, scenario_creator_kwargs={"num_scens": S},
       variable_probability=bad, _native_lib=emu, _device="cpu")
