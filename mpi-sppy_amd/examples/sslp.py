"""SSLP (stochastic server location), LP relaxation — workload C5a.

Restatement of ``examples/sslp/model/ReferenceModel.py`` + ``examples/sslp/sslp.py``
(reference) on the engine's LinearModel, binaries relaxed to [0, 1]:

  FacilityOpen[j] in [0,1] (j = 1..15, the ROOT nonants), Allocation[i,j] in [0,1],
  Dummy[j] >= 0;
  DemandConstraint[j]: sum_i Demand[i,j] Allocation[i,j] - Dummy[j] <= Capacity FacilityOpen[j]
  ClientConstraint[i]: sum_j Allocation[i,j] == ClientPresent[i]
  min sum_j FixedCost[j] FacilityOpen[j] + Penalty sum_j Dummy[j] - sum_{i,j} Revenue[i,j] Allocation[i,j]

Data: the deterministic parameters of sslp_15_45 (identical in every shipped scenario
file) and each shipped scenario's ClientPresent, extracted once from the reference's
.dat files into ``data/sslp_15_45.json`` (``scripts/make_sslp_data.py``).  Scenario
``ScenarioK`` of a shipped instance (``instance`` = 5, 10 or 15, or a ``data_dir``
ending in ``sslp_15_45_<n>/scenariodata`` as the reference passes) takes its shipped
ClientPresent; any other K draws ClientPresent[i] ~ Bernoulli(0.5) from
``RandomState(K)`` (the synthetic 10k-scenario workload).
Only the client rows' right-hand sides vary across scenarios.
"""
import json
import os
import re

import numpy as np

from .. import model as lm
from ..batch import BatchData, NonantSpec
from ..utils import sputils

_DATA = None


def data():
    global _DATA
    if _DATA is None:
        with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "sslp_15_45.json")) as f:
            _DATA = json.load(f)
    return _DATA


def _instance(data_dir, instance):
    if instance is not None:
        return str(instance)
    if data_dir is not None:
        m = re.search(r"sslp_\d+_\d+_(\d+)", data_dir)
        if m:
            return m.group(1)
    return None


def client_present(scennum, instance=None):
    """ClientPresent of scenario number K (1-based as the reference names them)."""
    d = data()
    shipped = d["ClientPresent"].get(instance) if instance is not None else None
    if shipped is not None and 1 <= scennum <= len(shipped):
        return np.array(shipped[scennum - 1], dtype=np.float64)
    rs = np.random.RandomState(scennum)
    return (rs.rand(d["NumClients"]) < 0.5).astype(np.float64)


def scenario_creator(scenario_name, data_dir=None, instance=None, num_scens=None):
    """One scenario (ReferenceModel.py + sslp.py:18-34), LP relaxation."""
    d = data()
    ns, nc = d["NumServers"], d["NumClients"]
    K = sputils.extract_num(scenario_name)
    present = client_present(K, _instance(data_dir, instance))
    m = lm.LinearModel(scenario_name)
    servers = list(range(1, ns + 1))
    clients = list(range(1, nc + 1))
    Open = m.add_indexed_var("FacilityOpen", servers, lb=0.0, ub=1.0)
    Alloc = m.add_indexed_var("Allocation", [(i, j) for i in clients for j in servers], lb=0.0, ub=1.0)
    Dummy = m.add_indexed_var("Dummy", servers, lb=0.0)
    for j in servers:
        m.add_constraint(lm.quicksum(d["Demand"][i - 1][j - 1] * Alloc[i, j] for i in clients) - Dummy[j]
                         - d["Capacity"] * Open[j], ub=0.0)
    for i in clients:
        m.add_constraint(lm.quicksum(Alloc[i, j] for j in servers), present[i - 1], present[i - 1])
    first = lm.quicksum(d["FixedCost"][j - 1] * Open[j] for j in servers)
    second = d["Penalty"] * lm.quicksum(Dummy[j] for j in servers) - lm.quicksum(
        d["Revenue"][i - 1][j - 1] * Alloc[i, j] for i in clients for j in servers)
    m.FirstStageCost = first
    m.set_objective(first + second, lm.minimize)
    m.FacilityOpen = Open
    sputils.attach_root_node(m, first, [Open])
    if num_scens is not None:
        m._mpisppy_probability = 1 / num_scens
    return m


def batch_creator(scenario_names, data_dir=None, instance=None, num_scens=None):
    """Vectorised: the same standard form for many scenarios (only the client rows'
    right-hand sides vary); tests/test_sslp.py checks it bit-exact against
    scenario_creator."""
    d = data()
    ns, nc = d["NumServers"], d["NumClients"]
    inst = _instance(data_dir, instance)
    S = len(scenario_names)
    n = ns + nc * ns + ns
    OPEN, ALLOC, DUMMY = 0, ns, ns + nc * ns

    def acol(i, j):           # Allocation[(i, j)] in (client, server) order, 0-based i, j
        return ALLOC + i * ns + j
    rowptr, colidx, vals = [0], [], []
    for j in range(ns):       # demand rows: columns sorted (Open_j < Alloc_.j < Dummy_j)
        cols = [(OPEN + j, -d["Capacity"])]
        cols += [(acol(i, j), d["Demand"][i][j]) for i in range(nc) if d["Demand"][i][j] != 0.0]
        cols += [(DUMMY + j, -1.0)]
        cols.sort()
        colidx += [c for c, _ in cols]
        vals += [v for _, v in cols]
        rowptr.append(len(colidx))
    for i in range(nc):       # client rows
        colidx += [acol(i, j) for j in range(ns)]
        vals += [1.0] * ns
        rowptr.append(len(colidx))
    m = len(rowptr) - 1
    P = np.stack([client_present(sputils.extract_num(nm), inst) for nm in scenario_names]) if S else \
        np.zeros((0, nc))
    BL = np.empty((S, m))
    BU = np.empty((S, m))
    BL[:, :ns] = -np.inf
    BU[:, :ns] = 0.0
    BL[:, ns:] = P
    BU[:, ns:] = P
    A = np.broadcast_to(np.asarray(vals, dtype=np.float64), (S, len(vals)))
    lb = np.zeros(n)
    ub = np.ones(n)
    ub[DUMMY:DUMMY + ns] = np.inf
    c = np.zeros(n)
    c[OPEN:OPEN + ns] = d["FixedCost"]
    c[DUMMY:DUMMY + ns] = d["Penalty"]
    for i in range(nc):
        for j in range(ns):
            c[acol(i, j)] = -d["Revenue"][i][j]
    c = np.where(c == 0.0, 0.0, c)
    names = ["FacilityOpen[%d]" % (j + 1) for j in range(ns)]
    names += ["Allocation[(%d, %d)]" % (i + 1, j + 1) for i in range(nc) for j in range(ns)]
    names += ["Dummy[%d]" % (j + 1) for j in range(ns)]
    nonant = NonantSpec(list(range(OPEN, OPEN + ns)), [1] * ns, list(range(ns)), [None], [np.ones(S)],
                        names[:ns])
    prob = [1 / num_scens if num_scens is not None else None] * S
    return BatchData(scenario_names, rowptr, colidx, A, BL, BU, lb, ub, c, 0.0, lm.minimize, prob, nonant,
                     names)


scenario_creator.batch_creator = batch_creator


def scenario_names_creator(num_scens, start=None):
    """ScenarioK, K from 1 (sslp.py:138-140)."""
    if start is None:
        start = 1
    return ["Scenario%d" % i for i in range(start, start + num_scens)]


def scenario_denouement(rank, scenario_name, scenario):
    pass
