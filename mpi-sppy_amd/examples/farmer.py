"""Scalable farmer (workloads C1-C3).

Restatement of ``examples/farmer/farmer.py`` (reference lines 26-250) on the
engine's LinearModel: same scenario naming (``scen<k>``; number scraped from the
right), same base/group split (k % 3, k // 3), same RandomState stream seeded
with ``k + seedoffset`` and drawn in CROPS insertion order for groups != 0
(farmer.py:62-73, 115-123, 177-183), same bounds, rows and costs.
``EnforceQuotas`` (0 <= QuantitySubQuotaSold <= PriceQuota) is a single-variable
row and is folded into the variable's bounds.

``scenario_creator.batch_creator`` builds the same standard form for many
scenarios at once (vectorised); ``tests/test_batch.py`` checks it bit-exact
against the per-scenario path.
"""
import numpy as np

from .. import model as lm
from ..batch import BatchData, NonantSpec
from ..utils import rng, sputils

_BASENAMES = ["BelowAverageScenario", "AverageScenario", "AboveAverageScenario"]
_YIELD = {
    "BelowAverageScenario": {"WHEAT": 2.0, "CORN": 2.4, "SUGAR_BEETS": 16.0},
    "AverageScenario": {"WHEAT": 2.5, "CORN": 3.0, "SUGAR_BEETS": 20.0},
    "AboveAverageScenario": {"WHEAT": 3.0, "CORN": 3.6, "SUGAR_BEETS": 24.0},
}
_PARMS = {
    "PriceQuota": {"WHEAT": 100000.0, "CORN": 100000.0, "SUGAR_BEETS": 6000.0},
    "SubQuotaSellingPrice": {"WHEAT": 170.0, "CORN": 150.0, "SUGAR_BEETS": 36.0},
    "SuperQuotaSellingPrice": {"WHEAT": 0.0, "CORN": 0.0, "SUGAR_BEETS": 10.0},
    "CattleFeedRequirement": {"WHEAT": 200.0, "CORN": 240.0, "SUGAR_BEETS": 0.0},
    "PurchasePrice": {"WHEAT": 238.0, "CORN": 210.0, "SUGAR_BEETS": 100000.0},
    "PlantingCostPerAcre": {"WHEAT": 150.0, "CORN": 230.0, "SUGAR_BEETS": 260.0},
}
_CROPBASE = ["WHEAT", "CORN", "SUGAR_BEETS"]


def _crops(cm):
    out = []
    for i in range(cm):
        out += ["WHEAT%d" % i, "CORN%d" % i, "SUGAR_BEETS%d" % i]
    return out


def _yields(scennum, cm, seedoffset, total_perturb, rel_perturb):
    """Yield of every crop, CROPS insertion order (farmer.py:159-183)."""
    base = _BASENAMES[scennum % 3]
    group = scennum // 3
    stream = np.random.RandomState()
    stream.seed(scennum + seedoffset)
    y = dict(_YIELD[base])
    if total_perturb != 0:
        for crop in y:
            y[crop] = y[crop] * (1 + total_perturb)
    if rel_perturb != 0:
        for crop in list(y):
            y[crop] = y[crop] * (1 + rel_perturb * stream.normal(0, 2))
    out = []
    for i in range(cm):
        for crop in _CROPBASE:
            v = y[crop]
            if group != 0:
                v = v + stream.rand()
            out.append(v)
    return out


def _yields_batch(nums, cm, seedoffset, total_perturb, rel_perturb):
    """(S, 3 cm) yields of many scenarios, == _yields row by row.  Without
    rel_perturb (no normal() draws) the per-scenario rand() streams come from the
    vectorised MT19937 (utils/rng.py: bit-exact RandomState(seed).rand()); with
    it, one RandomState per scenario as _yields."""
    nums = np.asarray(nums, dtype=np.int64)
    S = nums.size
    if rel_perturb != 0 or S == 0:
        return np.array([_yields(int(k), cm, seedoffset, total_perturb, rel_perturb) for k in nums]).reshape(S, 3 * cm)
    base = np.array([[_YIELD[_BASENAMES[b]][c] for c in _CROPBASE] for b in range(3)])   # [base][crop]
    if total_perturb != 0:
        base = base * (1 + total_perturb)
    Y = np.tile(base[nums % 3], (1, cm))                                                  # [S][i*3 + crop]
    draw = nums // 3 != 0
    if draw.any():
        Y[draw] = Y[draw] + rng.first_rands(nums[draw] + seedoffset, 3 * cm)
    return Y


def scenario_creator(scenario_name, use_integer=False, sense=lm.minimize, crops_multiplier=1,
                     num_scens=None, seedoffset=0, total_perturb=0, rel_perturb=0, relseed=0):
    """Build one farmer scenario (farmer.py:26-98 + 100-250)."""
    if use_integer:
        raise NotImplementedError("integer farmer (MIP subproblems) is outside the batched LP/QP engine")
    if sense not in (lm.minimize, lm.maximize):
        raise ValueError("Model sense Not recognized")
    scennum = sputils.extract_num(scenario_name)
    cm = crops_multiplier
    crops = _crops(cm)
    ylds = dict(zip(crops, _yields(scennum, cm, seedoffset, total_perturb, rel_perturb)))
    m = lm.LinearModel(_BASENAMES[scennum % 3] + str(scennum // 3))
    total_acreage = 500.0 * cm
    DA = m.add_indexed_var("DevotedAcreage", crops, lb=0.0, ub=total_acreage)
    QSub = m.add_indexed_var("QuantitySubQuotaSold", crops, lb=0.0)
    QSup = m.add_indexed_var("QuantitySuperQuotaSold", crops, lb=0.0)
    QP = m.add_indexed_var("QuantityPurchased", crops, lb=0.0)
    basename = {c: c.rstrip("0123456789") for c in crops}
    m.add_row([DA[c].index for c in crops], [1.0] * len(crops), ub=total_acreage)
    for c in crops:
        m.add_row([DA[c].index, QP[c].index, QSub[c].index, QSup[c].index],
                  [ylds[c], 1.0, -1.0, -1.0], lb=_PARMS["CattleFeedRequirement"][basename[c]])
    for c in crops:
        m.add_row([QSub[c].index, QSup[c].index, DA[c].index], [1.0, 1.0, -ylds[c]], ub=0.0)
    for c in crops:
        m.add_constraint(QSub[c], 0.0, _PARMS["PriceQuota"][basename[c]])
    first = lm.quicksum(_PARMS["PlantingCostPerAcre"][basename[c]] * DA[c] for c in crops)
    second = lm.quicksum(_PARMS["PurchasePrice"][basename[c]] * QP[c] for c in crops)
    second = second - lm.quicksum(_PARMS["SubQuotaSellingPrice"][basename[c]] * QSub[c] for c in crops)
    second = second - lm.quicksum(_PARMS["SuperQuotaSellingPrice"][basename[c]] * QSup[c] for c in crops)
    m.FirstStageCost = first
    if sense == lm.minimize:
        m.set_objective(first + second, lm.minimize)
    else:
        m.set_objective(-first - second, lm.maximize)
    m.DevotedAcreage = DA
    sputils.attach_root_node(m, first, [DA])
    if num_scens is not None:
        m._mpisppy_probability = 1 / num_scens
    return m


def batch_creator(scenario_names, use_integer=False, sense=lm.minimize, crops_multiplier=1,
                  num_scens=None, seedoffset=0, total_perturb=0, rel_perturb=0, relseed=0):
    """Vectorised: the standard form of many farmer scenarios at once."""
    if use_integer:
        raise NotImplementedError("integer farmer (MIP subproblems) is outside the batched LP/QP engine")
    S = len(scenario_names)
    cm = crops_multiplier
    crops = _crops(cm)
    nc = len(crops)
    n = 4 * nc
    DA, SUB, SUP, PUR = 0, nc, 2 * nc, 3 * nc
    Y = _yields_batch([sputils.extract_num(nm) for nm in scenario_names], cm, seedoffset, total_perturb,
                      rel_perturb)
    base = [c.rstrip("0123456789") for c in crops]
    # rows exactly as scenario_creator + LinearModel.add_row (columns sorted)
    rowptr = [0]
    colidx = []
    vals_const = []     # per nnz: value or None (yield)
    yield_of = []       # per nnz: crop index for yield entries, else -1
    colidx += list(range(DA, DA + nc)); vals_const += [1.0] * nc; yield_of += [-1] * nc
    rowptr.append(len(colidx))
    bl = [-np.inf]; bu = [500.0 * cm]
    for k in range(nc):   # feed: cols DA_k, SUB_k, SUP_k, PUR_k (sorted)
        colidx += [DA + k, SUB + k, SUP + k, PUR + k]
        vals_const += [None, -1.0, -1.0, 1.0]
        yield_of += [k, -1, -1, -1]
        rowptr.append(len(colidx))
        bl.append(_PARMS["CattleFeedRequirement"][base[k]]); bu.append(np.inf)
    for k in range(nc):   # limit: cols DA_k, SUB_k, SUP_k
        colidx += [DA + k, SUB + k, SUP + k]
        vals_const += [None, 1.0, 1.0]
        yield_of += [k, -1, -1]
        rowptr.append(len(colidx))
        bl.append(-np.inf); bu.append(0.0)
    nnz = len(colidx)
    A = np.empty((S, nnz))
    sign = {}
    for p in range(nnz):
        if yield_of[p] < 0:
            A[:, p] = vals_const[p]
    # feed rows: +yield ; limit rows: -yield
    p = nc
    for k in range(nc):
        A[:, p] = Y[:, k]
        p += 4
    for k in range(nc):
        A[:, p] = -Y[:, k]
        p += 3
    lb = np.zeros(n)
    ub = np.full(n, np.inf)
    ub[DA:DA + nc] = 500.0 * cm
    for k in range(nc):
        ub[SUB + k] = _PARMS["PriceQuota"][base[k]]
    c = np.zeros(n)
    for k in range(nc):
        c[DA + k] = _PARMS["PlantingCostPerAcre"][base[k]]
        c[PUR + k] = _PARMS["PurchasePrice"][base[k]]
        c[SUB + k] = -_PARMS["SubQuotaSellingPrice"][base[k]]
        c[SUP + k] = -_PARMS["SuperQuotaSellingPrice"][base[k]]
    if sense == lm.maximize:
        c = -c
    c = np.where(c == 0.0, 0.0, c)   # normalise -0.0 the way LinExpr coefficients add up
    order = sorted(range(nc), key=lambda k: crops[k])
    names = []
    for fam in ["DevotedAcreage", "QuantitySubQuotaSold", "QuantitySuperQuotaSold", "QuantityPurchased"]:
        names += ["%s[%s]" % (fam, cr) for cr in crops]
    nonant = NonantSpec([DA + k for k in order], [1] * nc, list(range(nc)), [None], [np.ones(S)],
                        [names[DA + k] for k in order])
    prob = [1 / num_scens if num_scens is not None else None] * S
    return BatchData(scenario_names, rowptr, colidx, A, bl, bu, lb, ub, c, 0.0, sense, prob,
                     nonant, names)


scenario_creator.batch_creator = batch_creator


def scenario_names_creator(num_scens, start=None):
    if start is None:
        start = 0
    return ["scen%d" % i for i in range(start, start + num_scens)]


def kw_creator(options):
    return {"use_integer": options.get("use_integer", False),
            "crops_multiplier": options.get("crops_multiplier", 1),
            "num_scens": options.get("num_scens", None)}


def scenario_denouement(rank, scenario_name, scenario):
    pass
