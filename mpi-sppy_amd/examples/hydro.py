"""hydro (elec3) three-stage hydro-thermal scheduling LP — the reference's multistage PH pin.

Restatement of ``mpisppy/tests/examples/hydro/hydro.py`` (reference) on the engine's
LinearModel.  Per stage t = 1..3: thermal Pgt[t] in [PgtMin, PgtMax], hydro Pgh[t] in
[PghMin, PghMax], unserved PDns[t] in [0, D[t]], reservoir Vol[t] in [VMin, VMax], a free
StageCost[t]; one final slack sl >= 0 (hydro.py:74-94).  Rows (hydro.py:106-136):

  StageCost[t] == r[t] (betaGt Pgt[t] + betaGh Pgh[t] + betaDns PDns[t])  (+ sl at t = 3)
  Pgt[t] + Pgh[t] + PDns[t] - D[t] == 0                                   (demand)
  Vol[t] - Vol[t-1] <= u[t] (A[t] - Pgh[t])          (Vol[0] = V0)        (conserv)
  sl >= 4166.67 (V0 - Vol[3])                                             (fcfe)

with r[t] = (1/1.1)^(duracion[t]/T) (discount_rule, hydro.py:96-99) and the objective
sum_t StageCost[t].  Tree (MakeNodesforScen, hydro.py:183-210): ROOT holds
[Pgt[1], Pgh[1], PDns[1], Vol[1]], stage-2 node ``ROOT_<(snum-1)//BF[0]>`` (cond_prob
1/BF[0]) holds the same four of stage 2; scenario names are ``Scen1..Scen9`` (one-based)
and probabilities are left uniform.  Data: the nine shipped scenario files (only the
inflows A[2], A[3] differ), extracted once into ``data/hydro.json``
(``scripts/make_hydro_data.py``).
"""
import json
import os

from .. import model as lm
from ..scenario_tree import ScenarioNode
from ..utils import sputils

_DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "hydro.json")
_cache = {}


def _scenario_data(scenario_name):
    if "d" not in _cache:
        with open(_DATA) as f:
            _cache["d"] = json.load(f)["scenarios"]
    d = _cache["d"]
    if scenario_name not in d:
        raise ValueError("hydro: no data for scenario %s (shipped: Scen1..Scen9)" % scenario_name)
    return d[scenario_name]


def hydro_model_creator(p, name=None):
    """The elec3 LP of one scenario's parameters ``p`` (hydro.py:31-144)."""
    T = int(p["nb_etap"])
    m = lm.LinearModel(name)
    etap = list(range(1, T + 1))
    Pgt = m.add_indexed_var("Pgt", etap, p["PgtMin"], p["PgtMax"])
    Pgh = m.add_indexed_var("Pgh", etap, p["PghMin"], p["PghMax"])
    PDns = m.add_indexed_var("PDns", etap, 0.0, None)
    for t in etap:
        PDns[t].ub = p["D"][str(t)]
    Vol = m.add_indexed_var("Vol", etap, p["VMin"], p["VMax"])
    sl = m.add_var("sl", 0.0, None)
    StageCost = m.add_indexed_var("StageCost", etap, None, None)
    r = {t: (1 / 1.1) ** (p["duracion"][str(t)] / float(p["T"])) for t in etap}
    for t in etap:
        e = StageCost[t] - r[t] * (p["betaGt"] * Pgt[t] + p["betaGh"] * Pgh[t] + p["betaDns"] * PDns[t])
        if t == T:
            e = e - sl
        m.add_constraint(e, 0.0, 0.0)
    for t in etap:
        m.add_constraint(Pgt[t] + Pgh[t] + PDns[t] - p["D"][str(t)], 0.0, 0.0)
    for t in etap:
        u, A = p["u"][str(t)], p["A"][str(t)]
        prev = p["V0"] if t == 1 else Vol[t - 1]
        m.add_constraint(Vol[t] - prev + u * Pgh[t], None, u * A)
    m.add_constraint(sl - 4166.67 * (p["V0"] - Vol[3]), 0.0, None)
    m.set_objective(lm.quicksum(StageCost[t] for t in etap), lm.minimize)
    m.Pgt, m.Pgh, m.PDns, m.Vol, m.sl, m.StageCost = Pgt, Pgh, PDns, Vol, sl, StageCost
    return m


def MakeNodesforScen(model, BFs, scennum):
    """hydro.py:183-210 (scennum is one-based)."""
    ndn = "ROOT_" + str((scennum - 1) // BFs[0])
    return [ScenarioNode("ROOT", 1.0, 1, model.StageCost[1],
                         [model.Pgt[1], model.Pgh[1], model.PDns[1], model.Vol[1]], model),
            ScenarioNode(ndn, 1.0 / BFs[0], 2, model.StageCost[2],
                         [model.Pgt[2], model.Pgh[2], model.PDns[2], model.Vol[2]], model,
                         parent_name="ROOT")]


def scenario_creator(scenario_name, branching_factors=None, data_path=None):
    """hydro.py:213-236: ``data_path`` is accepted for the reference's signature;
    the data come from the packaged extract."""
    if branching_factors is None:
        raise ValueError("Hydro scenario_creator requires branching_factors")
    snum = sputils.extract_num(scenario_name)
    model = hydro_model_creator(_scenario_data(scenario_name), name=scenario_name)
    model._mpisppy_node_list = MakeNodesforScen(model, branching_factors, snum)
    return model


def scenario_denouement(rank, scenario_name, scenario):
    pass


def scenario_names_creator(num_scens, start=None):
    start = 1 if start is None else start
    return ["Scen%d" % k for k in range(start, start + num_scens)]
