"""Network design (netdes), LP relaxation — workload C5b.

Restatement of the reference's ``examples/netdes/netdes.py:17-87`` on the engine's
LinearModel, first-stage binaries relaxed to [0, 1]:

  x[e] in [0,1] (build edge e; the ROOT nonants, ``model.x[:,:]``), y[e] >= 0 (flow);
  vubs[e]:  y[e] - u[e] x[e] <= 0                                 (netdes.py:56-60)
  bals[i]:  sum_{(i,j)} y[i,j] - sum_{(j,i)} y[j,i] == b[i]      (netdes.py:62-69)
  min sum_e c[e] x[e] + sum_e d[e] y[e]                           (netdes.py:50-54)

Edges are the nonzeros of the adjacency matrix in row-major order (parse.py:58-59).
Data: the reference's .dat instances, extracted once into
``data/netdes_<instance>.npz`` (``scripts/make_netdes_data.py``).  The reference takes
the instance through ``path`` (RuntimeError without it, netdes.py:18-21); here ``path``
may name the reference's .dat file (its basename selects the extracted data) or
``instance`` names it directly.  Scenario indices are zero-based and stripped from the
right of the name (``_get_scenario_ix``, netdes.py:79-87).  A shipped scenario k < K
takes its own (d, u, b) and probability p[k] (parse.py:32-45); any other k (the
synthetic 10k-scenario workload) takes shipped scenario k mod K with
its flow costs d scaled by 1 + 0.2 (r - 1/2), r ~ RandomState(k).rand(E), and
probability 1/num_scens (only with num_scens given: without it an index k >= K raises
the reference's ValueError, parse.py:34-37).  Varying per scenario: the vubs' u coefficients, the cost
vector (d), the bals right-hand sides (b).
"""
import os

import numpy as np

from .. import model as lm
from ..batch import BatchData, NonantSpec
from ..utils import sputils

_DATA = {}
DEFAULT_INSTANCE = "network-10-10-H-01"


def data(instance=DEFAULT_INSTANCE):
    if instance not in _DATA:
        f = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "netdes_%s.npz" % instance)
        if not os.path.exists(f):
            raise RuntimeError("netdes instance %s is not among the extracted data files" % instance)
        with np.load(f) as z:
            _DATA[instance] = {k: z[k] for k in z.files}
    return _DATA[instance]


def _instance(path, instance):
    if instance is not None:
        return instance
    if path is None:
        raise RuntimeError("Must provide the name of the .dat file containing the instance data via the "
                           "path argument to scenario_creator")
    return os.path.splitext(os.path.basename(path))[0]


def _get_scenario_ix(sname):
    """netdes.py:79-87: the digits at the right end of the name."""
    i = len(sname) - 1
    while i > 0 and sname[i - 1].isdigit():
        i -= 1
    return int(sname[i:])


def scenario_data(k, instance=DEFAULT_INSTANCE, synthetic=False):
    """(d, u, b, p) of scenario index k (p None for a synthetic scenario).  Indices
    beyond the instance's K scenarios exist only in the synthetic workload
    (``synthetic``, i.e. num_scens given); otherwise they raise the reference's
    ValueError (parse.py:34-37)."""
    z = data(instance)
    K = len(z["p"])
    if k < 0 or (k >= K and not synthetic):
        raise ValueError("Provided scenario index ({}) could not be found ({} total scenarios)".format(k, K))
    if k < K:
        return z["d"][k], z["u"][k], z["b"][k], float(z["p"][k])
    r = np.random.RandomState(k).rand(len(z["c"]))
    return z["d"][k % K] * (1.0 + 0.2 * (r - 0.5)), z["u"][k % K], z["b"][k % K], None


def scenario_creator(scenario_name, path=None, instance=None, num_scens=None):
    """One scenario (netdes.py:17-71), LP relaxation."""
    inst = _instance(path, instance)
    z = data(inst)
    k = _get_scenario_ix(scenario_name)
    d, u, b, p = scenario_data(k, inst, synthetic=num_scens is not None)
    edges = [(int(i), int(j)) for i, j in z["edges"]]
    m = lm.LinearModel(scenario_name)
    x = m.add_indexed_var("x", edges, lb=0.0, ub=1.0)
    y = m.add_indexed_var("y", edges, lb=0.0)
    for e, ij in enumerate(edges):
        m.add_constraint(y[ij] - u[e] * x[ij], ub=0.0)
    for i in range(int(z["N"])):
        out_nbs = [ij for ij in edges if ij[0] == i]
        in_nbs = [ij for ij in edges if ij[1] == i]
        lhs = lm.quicksum(y[ij] for ij in out_nbs) - lm.quicksum(y[ij] for ij in in_nbs)
        m.add_constraint(lhs, b[i], b[i])
    first = lm.quicksum(z["c"][e] * x[ij] for e, ij in enumerate(edges))
    second = lm.quicksum(d[e] * y[ij] for e, ij in enumerate(edges))
    m.FirstStageCost = first
    m.set_objective(first + second, lm.minimize)
    m.x = x
    sputils.attach_root_node(m, first, [x])
    if num_scens is not None:
        m._mpisppy_probability = 1 / num_scens
    elif p is not None:
        m._mpisppy_probability = p
    return m


def batch_creator(scenario_names, path=None, instance=None, num_scens=None):
    """Vectorised: the same standard form for many scenarios; tests/test_netdes.py
    checks it bit-exact against scenario_creator."""
    inst = _instance(path, instance)
    z = data(inst)
    N, ed = int(z["N"]), z["edges"]
    E = len(ed)
    S = len(scenario_names)
    n = 2 * E
    rowptr, colidx = [0], []
    for e in range(E):                               # vubs: x_e (col e) < y_e (col E + e)
        colidx += [e, E + e]
        rowptr.append(len(colidx))
    row_sign = []
    for i in range(N):                               # bals: y columns in edge order
        es = [e for e in range(E) if ed[e, 0] == i or ed[e, 1] == i]
        colidx += [E + e for e in es]
        row_sign.append([1.0 if ed[e, 0] == i else -1.0 for e in es])
        rowptr.append(len(colidx))
    m = E + N
    A = np.empty((S, len(colidx)))
    c = np.empty((S, n))
    BL = np.empty((S, m))
    BU = np.empty((S, m))
    bal_vals = np.concatenate(row_sign) if row_sign else np.zeros(0)
    prob = []
    for s, nm in enumerate(scenario_names):
        d, u, b, p = scenario_data(_get_scenario_ix(nm), inst, synthetic=num_scens is not None)
        A[s, 0:2 * E:2] = -u
        A[s, 1:2 * E:2] = 1.0
        A[s, 2 * E:] = bal_vals
        c[s, :E] = z["c"]
        c[s, E:] = d
        BL[s, :E] = -np.inf
        BU[s, :E] = 0.0
        BL[s, E:] = b
        BU[s, E:] = b
        prob.append(1 / num_scens if num_scens is not None else p)
    lb = np.zeros(n)
    ub = np.concatenate([np.ones(E), np.full(E, np.inf)])
    names = ["x[%s]" % ((int(i), int(j)),) for i, j in ed] + ["y[%s]" % ((int(i), int(j)),) for i, j in ed]
    nonant = NonantSpec(list(range(E)), [1] * E, list(range(E)), [None], [np.ones(S)], names[:E])
    return BatchData(scenario_names, rowptr, colidx, A, BL, BU, lb, ub, c, 0.0, lm.minimize, prob, nonant, names)


scenario_creator.batch_creator = batch_creator


def scenario_names_creator(num_scens, start=None):
    """Scenario0.. (zero-based, netdes.py:7)."""
    if start is None:
        start = 0
    return ["Scenario%d" % i for i in range(start, start + num_scens)]


def scenario_denouement(rank, scenario_name, scenario):
    pass
