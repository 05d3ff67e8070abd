"""aircond multistage production planning (workload C4).

Restatement of ``mpisppy/tests/examples/aircond.py`` (reference lines 19-329):
per-node demands drawn from a RandomState seeded with
``start_seed + node_idx(path)`` and clipped to [min_d, max_d]
(``_demands_creator`` 37-67), one stage block of five variables per stage
(``_StageModel_creator`` 88-184), material balance rows (214-224) and the node
list of ``MakeNodesforScen`` (251-301): nonants [RegularProd, OvertimeProd] per
non-leaf stage, cond_prob 1/branching_factors[stage-2].  ``start_ups`` (binary)
and ``QuadShortCoeff > 0`` are not supported (MIP / quadratic second stage).
"""
import numpy as np

from .. import model as lm
from ..batch import BatchData, NonantSpec
from ..scenario_tree import ScenarioNode
from ..utils import sputils

parms = {"mu_dev": 0.0, "sigma_dev": 40.0, "start_ups": False, "StartUpCost": 300.0,
         "start_seed": 1134, "min_d": 0.0, "max_d": 400.0, "starting_d": 200.0,
         "BeginInventory": 200.0, "InventoryCost": 0.5, "LastInventoryCost": -0.8,
         "Capacity": 200.0, "RegularProdCost": 1.0, "OvertimeProdCost": 3.0,
         "NegInventoryCost": 5.0, "QuadShortCoeff": 0.0}


def _kw(kwargs, name):
    return kwargs.get(name, parms[name])


def _path(sname, branching_factors):
    scennum = sputils.extract_num(sname)
    prod = int(np.prod(branching_factors))
    s = int(scennum % prod)
    nodenames = ["ROOT"]
    for bf in branching_factors:
        prod = prod // bf
        nodenames.append(str(s // prod))
        s = s % prod
    return nodenames


def _demands_creator(sname, sample_branching_factors, root_name="ROOT", **kwargs):
    """aircond.py:37-67 (the per-node seeded demand walk)."""
    if "start_seed" not in kwargs:
        raise RuntimeError("start_seed not in kwargs=%s" % kwargs)
    start_seed = kwargs["start_seed"]
    max_d = kwargs.get("max_d", 400)
    min_d = kwargs.get("min_d", 0)
    mu_dev = kwargs.get("mu_dev", parms["mu_dev"])
    sigma_dev = kwargs.get("sigma_dev", parms["sigma_dev"])
    branching_factors = sample_branching_factors
    nodenames = _path(sname, branching_factors)
    d = kwargs.get("starting_d", 200)
    demands = [d]
    stagelist = [int(x) for x in nodenames[1:]]
    stream = np.random.RandomState()
    for t in range(1, len(nodenames)):
        stream.seed(start_seed + sputils.node_idx(stagelist[:t], branching_factors))
        d = min(max_d, max(min_d, d + stream.normal(mu_dev, sigma_dev)))
        demands.append(d)
    return demands, nodenames


def _check_kwargs(kwargs):
    if _kw(kwargs, "start_ups"):
        raise NotImplementedError("aircond start_ups (binary StartUp) is outside the LP/QP engine")
    if _kw(kwargs, "QuadShortCoeff") > 0:
        raise NotImplementedError("aircond QuadShortCoeff > 0 (quadratic second stage) not supported")


def aircond_model_creator(demands, **kwargs):
    """aircond.py:188-249 as a LinearModel (vars stage by stage, then rows)."""
    _check_kwargs(kwargs)
    m = lm.LinearModel()
    T = len(demands)
    if T > 25:
        raise RuntimeError("The number of stages exceeds 25")
    bigM = _kw(kwargs, "Capacity") * 25
    st = []
    for t in range(1, T + 1):
        v = {}
        v["RegularProd"] = m.add_var("stage_model_%d.RegularProd" % t, 0.0, bigM)
        v["OvertimeProd"] = m.add_var("stage_model_%d.OvertimeProd" % t, 0.0, bigM)
        v["Inventory"] = m.add_var("stage_model_%d.Inventory" % t, -bigM, bigM)
        v["negInventory"] = m.add_var("stage_model_%d.negInventory" % t, 0.0, bigM)
        v["posInventory"] = m.add_var("stage_model_%d.posInventory" % t, 0.0, bigM)
        m.add_constraint(v["RegularProd"], None, _kw(kwargs, "Capacity"))       # MaximumCapacity
        m.add_constraint(v["Inventory"] - v["posInventory"] + v["negInventory"], 0.0, 0.0)  # dole
        st.append(v)
    for t in range(1, T + 1):
        v = st[t - 1]
        if t == 1:
            e = _kw(kwargs, "BeginInventory") + v["RegularProd"] + v["OvertimeProd"] - v["Inventory"]
        else:
            e = st[t - 2]["Inventory"] + v["RegularProd"] + v["OvertimeProd"] - v["Inventory"]
        m.add_constraint(e, demands[t - 1], demands[t - 1])
    obj = lm.LinExpr()
    for t in range(1, T + 1):
        v = st[t - 1]
        last = (t == T)
        inv = _kw(kwargs, "LastInventoryCost") if last else _kw(kwargs, "InventoryCost")
        stage_cost = (_kw(kwargs, "RegularProdCost") * v["RegularProd"]
                      + _kw(kwargs, "OvertimeProdCost") * v["OvertimeProd"]
                      + inv * v["posInventory"] + _kw(kwargs, "NegInventoryCost") * v["negInventory"])
        v["StageObjective"] = stage_cost
        obj = obj + stage_cost
    m.set_objective(obj, lm.minimize)
    m.stage_models = st
    m.T = list(range(1, T + 1))
    return m


def MakeNodesforScen(model, nodenames, branching_factors, starting_stage=1):
    """aircond.py:251-301."""
    nodes = []
    ndn = None
    for stage in model.T:
        v = model.stage_models[stage - 1]
        nonant_list = [v["RegularProd"], v["OvertimeProd"]]
        suppl = [v["Inventory"]]
        if stage == 1:
            ndn = "ROOT"
            nodes.append(ScenarioNode(ndn, 1.0, stage, v["StageObjective"], nonant_list, model,
                                      nonant_ef_suppl_list=suppl))
        elif stage <= starting_stage:
            parent = ndn
            ndn = parent + "_0"
            nodes.append(ScenarioNode(ndn, 1.0, stage, v["StageObjective"], nonant_list, model,
                                      nonant_ef_suppl_list=suppl, parent_name=parent))
        elif stage < max(model.T):
            parent = ndn
            ndn = parent + "_" + nodenames[stage - starting_stage]
            nodes.append(ScenarioNode(ndn, 1.0 / branching_factors[stage - starting_stage - 1], stage,
                                      v["StageObjective"], nonant_list, model,
                                      nonant_ef_suppl_list=suppl, parent_name=parent))
    return nodes


def scenario_creator(sname, **kwargs):
    if "start_seed" not in kwargs:
        kwargs["start_seed"] = parms["start_seed"]
    if "branching_factors" not in kwargs:
        raise RuntimeError("scenario_creator for aircond needs branching_factors in kwargs")
    bfs = kwargs["branching_factors"]
    demands, nodenames = _demands_creator(sname, bfs, root_name="ROOT", **kwargs)
    model = aircond_model_creator(demands, **kwargs)
    model._mpisppy_node_list = MakeNodesforScen(model, nodenames, bfs)
    model._mpisppy_probability = 1 / np.prod(bfs)
    return model


def batch_creator(scenario_names, **kwargs):
    """Vectorised aircond: same arrays as scenario_creator, demands cached per node."""
    if "start_seed" not in kwargs:
        kwargs["start_seed"] = parms["start_seed"]
    _check_kwargs(kwargs)
    bfs = kwargs["branching_factors"]
    S = len(scenario_names)
    T = len(bfs) + 1
    # template from one scenario: the pattern is demand-independent
    tmpl = aircond_model_creator([0.0] * T, **kwargs)
    f = tmpl.standard_form()
    m = len(f["bl"])
    cache = {}
    start_seed = kwargs["start_seed"]
    max_d = kwargs.get("max_d", 400)
    min_d = kwargs.get("min_d", 0)
    mu_dev = kwargs.get("mu_dev", parms["mu_dev"])
    sigma_dev = kwargs.get("sigma_dev", parms["sigma_dev"])
    starting_d = kwargs.get("starting_d", 200)
    stream = np.random.RandomState()
    D = np.empty((S, T))
    paths = []
    for k, nm in enumerate(scenario_names):
        nodenames = _path(nm, bfs)
        paths.append(nodenames)
        stagelist = [int(x) for x in nodenames[1:]]
        d = starting_d
        D[k, 0] = d
        for t in range(1, T):
            key = tuple(stagelist[:t])
            if key not in cache:
                stream.seed(start_seed + sputils.node_idx(stagelist[:t], bfs))
                cache[key] = stream.normal(mu_dev, sigma_dev)
            d = min(max_d, max(min_d, d + cache[key]))
            D[k, t] = d
    bl = np.broadcast_to(f["bl"], (S, m)).copy()
    bu = np.broadcast_to(f["bu"], (S, m)).copy()
    # material-balance rows are the last T rows; rhs = demand (minus BeginInventory at t=1)
    beg = _kw(kwargs, "BeginInventory")
    for t in range(T):
        r = m - T + t
        rhs = D[:, t] - (beg if t == 0 else 0.0)
        bl[:, r] = rhs
        bu[:, r] = rhs
    A = np.broadcast_to(f["vals"], (S, len(f["vals"]))).copy()
    slot_col, slot_stage, slot_local, vnames = [], [], [], []
    for t in range(1, T):
        for i, nmv in enumerate(["RegularProd", "OvertimeProd"]):
            slot_col.append(tmpl.stage_models[t - 1][nmv].index)
            slot_stage.append(t)
            slot_local.append(i)
            vnames.append(tmpl.stage_models[t - 1][nmv].name)
    node_names = [None]
    cond_prob = [np.ones(S)]
    for t in range(2, T):
        names_t = []
        for p in paths:
            ndn = "ROOT"
            for u in range(2, t + 1):
                ndn = ndn + "_" + p[u - 1]
            names_t.append(ndn)
        node_names.append(names_t)
        cond_prob.append(np.full(S, 1.0 / bfs[t - 2]))
    nonant = NonantSpec(slot_col, slot_stage, slot_local, node_names, cond_prob, vnames)
    prob = [1 / np.prod(bfs)] * S
    return BatchData(scenario_names, f["rowptr"], f["colidx"], A, bl, bu, f["lb"], f["ub"], f["c"],
                     f["c0"], f["sense"], prob, nonant, [v.name for v in tmpl._vars])


scenario_creator.batch_creator = batch_creator


def kw_creator(options):
    """All model parameters with the reference defaults (aircond.py:19-35), as
    the reference's kw_creator supplies them."""
    kw = {k: options.get(k, v) for k, v in parms.items()}
    kw["branching_factors"] = options.get("branching_factors")
    return kw


def scenario_names_creator(num_scens, start=None):
    if start is None:
        start = 0
    return ["scen%d" % i for i in range(start, start + num_scens)]
