"""Scenario generators and batch extraction (CPU): bit-exact data and nonant maps."""
import numpy as np
import pytest

import mpisppy_amd  # noqa: F401
from mpisppy_amd import batch as bm
from mpisppy_amd.examples import aircond, farmer
from mpisppy_amd.utils import sputils
from oracle import models as om


def _same(a, b):
    for k in ["rowptr", "colidx", "A_full", "bl", "bu", "lb", "ub", "c", "c0"]:
        x, y = getattr(a, k), getattr(b, k)
        x = np.asarray(x)
        y = np.asarray(y)
        if x.ndim != y.ndim:   # shared vs per-scenario representation
            x = np.broadcast_to(x, y.shape) if x.ndim < y.ndim else x
            y = np.broadcast_to(y, x.shape) if y.ndim < x.ndim else y
        assert np.array_equal(x, y), k
    assert np.array_equal(a.nonant.slot_col, b.nonant.slot_col)
    assert np.array_equal(a.nonant.slot_stage, b.nonant.slot_stage)
    assert np.array_equal(a.nonant.slot_local, b.nonant.slot_local)
    assert a.nonant.var_names == b.nonant.var_names


# 40 and 110: the vectorised yields draw 6 cm words per scenario, past the 227
# of the first half-twist (40) and past one whole 624-word twist (110)
@pytest.mark.parametrize("cm", [1, 2, 11, 40, 110])
def test_farmer_batch_equals_models(cm):
    names = farmer.scenario_names_creator(20)
    kw = {"crops_multiplier": cm, "num_scens": 20}
    models = [farmer.scenario_creator(n, **kw) for n in names]
    _same(farmer.batch_creator(names, **kw), bm.from_models(names, models))


@pytest.mark.parametrize("k", [1, 227, 228, 623, 624, 625, 1300])
def test_rng_first_rands_any_length(k):
    """utils/rng.py against numpy's own legacy RandomState, across twist boundaries."""
    from mpisppy_amd.utils import rng
    seeds = np.array([0, 1, 7, 12345, 2 ** 32 - 1])
    got = rng.first_rands(seeds, k)
    for i, sd in enumerate(seeds):
        assert np.array_equal(got[i], np.random.RandomState(int(sd)).rand(k))


def test_farmer_nonant_order_string_sort():
    """DevotedAcreage keys sorted as strings (scenario_tree.py:39): CORN0, CORN1, CORN10, CORN2..."""
    b = farmer.batch_creator(["scen0"], crops_multiplier=11)
    names = [v.split("[")[1][:-1] for v in b.nonant.var_names]
    assert names[:4] == ["CORN0", "CORN1", "CORN10", "CORN2"]
    assert names == sorted(names)
    b1 = farmer.batch_creator(["scen0"])
    assert b1.nonant.var_names[1] == "DevotedAcreage[SUGAR_BEETS0]"   # test_w_writer.py:107


def test_farmer_yields_match_oracle():
    """Yield coefficients identical to the oracle's independent restatement (farmer.py:177-183)."""
    names = farmer.scenario_names_creator(40)
    b = farmer.batch_creator(names, num_scens=40, crops_multiplier=2)
    for k, n in enumerate(names):
        o = om.farmer(n, crops_multiplier=2, num_scens=40)
        A = b.scenario_A(k)
        # compare the yield entries: the oracle's feed rows hold +yield on DA columns
        y_ref = np.array([o.A[1 + c, c] for c in range(6)])
        y_got = np.array([A[1 + c, c] for c in range(6)])
        assert np.array_equal(y_ref, y_got)


def test_aircond_batch_equals_models():
    bfs = [3, 3, 2]
    names = ["scen%d" % i for i in range(18)]
    kw = {"branching_factors": bfs, "start_seed": 0}
    models = [aircond.scenario_creator(n, **kw) for n in names]
    a = aircond.batch_creator(names, **kw)
    b = bm.from_models(names, models)
    _same(a, b)
    for t in range(1, a.nonant.nstages):
        assert a.nonant.node_names[t] == b.nonant.node_names[t]
        assert np.array_equal(a.nonant.cond_prob[t], b.nonant.cond_prob[t])


def test_aircond_demands_match_oracle():
    bfs = [4, 3, 2]
    for i in range(24):
        d1, n1 = aircond._demands_creator("scen%d" % i, bfs, start_seed=0)
        d2, n2 = om.aircond_demands("scen%d" % i, bfs, start_seed=0)
        assert d1 == d2 and n1 == n2


def test_compress_invariant_and_varying():
    names = farmer.scenario_names_creator(9)
    b = farmer.batch_creator(names, num_scens=9).compress()
    assert b.nvar == 6                    # the 6 yield entries vary (groups >= 1)
    assert not b.c_vary and not b.bnd_vary and not b.rhs_vary
    for k in range(9):
        assert np.array_equal(b.scenario_A(k), farmer.batch_creator([names[k]], num_scens=9).scenario_A(0))


def test_rank_slices_reference_rule():
    """contiguous slices, range(int(r*S/R), int((r+1)*S/R)) (sputils.py:803-810)."""
    assert sputils.rank_slices(10, 3) == [[0, 1, 2], [3, 4, 5], [6, 7, 8, 9]]
    assert sputils.rank_bounds(100000, 8)[3] == (37500, 50000)
    assert sputils.create_nodenames_from_branching_factors([2, 2])[:3] == ["ROOT", "ROOT_0", "ROOT_1"]


def test_pattern_mismatch_raises():
    m1 = farmer.scenario_creator("scen0", num_scens=2)
    m2 = farmer.scenario_creator("scen1", num_scens=2, crops_multiplier=2)
    with pytest.raises(RuntimeError):
        bm.from_models(["scen0", "scen1"], [m1, m2])
