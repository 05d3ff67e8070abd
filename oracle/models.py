"""Oracle scenario models (dense standard form) — TEST INFRASTRUCTURE ONLY.

Independent restatements of the reference's scenario creators, written
directly as dense LP standard form  min c'x + c0, bl <= Ax <= bu, lb <= x <= ub:

* farmer      — ``examples/farmer/farmer.py:26-250`` (scalable, RandomState
                seeded with the scenario number, yields perturbed in CROPS
                insertion order for groups != 0, lines 62-73, 115-123, 177-183)
* docs farmer — ``doc/src/examples.rst:56-94, 175-190`` (good/average/bad)
* aircond     — ``mpisppy/tests/examples/aircond.py:37-67, 88-329``
                (per-node seeded demands via ``sputils.node_idx``)

Nonant order follows ``scenario_tree.build_vardatalist`` (``scenario_tree.py:11-42``):
indexed Vars are expanded in ``sorted(keys)`` (string sort for farmer),
scalar Vars keep the given order.
"""
import os
import re
import numpy as np

INF = np.inf


def extract_num(name):
    """``sputils.extract_num`` (``utils/sputils.py:481-490``)."""
    return int(re.compile(r"(\d+)$").search(name).group(1))


class Scen:
    """One scenario in dense standard form plus its scenario-tree node list."""

    def __init__(self, name, var_names, c, c0, A, bl, bu, lb, ub, nodes, prob):
        self.name = name
        self.var_names = list(var_names)
        self.c = np.asarray(c, dtype=np.float64)
        self.c0 = float(c0)
        self.A = np.asarray(A, dtype=np.float64)
        self.bl = np.asarray(bl, dtype=np.float64)
        self.bu = np.asarray(bu, dtype=np.float64)
        self.lb = np.asarray(lb, dtype=np.float64)
        self.ub = np.asarray(ub, dtype=np.float64)
        # nodes: list of (node_name, cond_prob, stage, [var index ...])
        self.nodes = nodes
        self.prob = prob


# ---------------------------------------------------------------- farmer
_FARMER_BASE = ["BelowAverageScenario", "AverageScenario", "AboveAverageScenario"]
_FARMER_YIELD = {
    "BelowAverageScenario": {"WHEAT": 2.0, "CORN": 2.4, "SUGAR_BEETS": 16.0},
    "AverageScenario": {"WHEAT": 2.5, "CORN": 3.0, "SUGAR_BEETS": 20.0},
    "AboveAverageScenario": {"WHEAT": 3.0, "CORN": 3.6, "SUGAR_BEETS": 24.0},
}
_FARMER_DATA = {
    "PriceQuota": {"WHEAT": 100000.0, "CORN": 100000.0, "SUGAR_BEETS": 6000.0},
    "SubQuotaSellingPrice": {"WHEAT": 170.0, "CORN": 150.0, "SUGAR_BEETS": 36.0},
    "SuperQuotaSellingPrice": {"WHEAT": 0.0, "CORN": 0.0, "SUGAR_BEETS": 10.0},
    "CattleFeedRequirement": {"WHEAT": 200.0, "CORN": 240.0, "SUGAR_BEETS": 0.0},
    "PurchasePrice": {"WHEAT": 238.0, "CORN": 210.0, "SUGAR_BEETS": 100000.0},
    "PlantingCostPerAcre": {"WHEAT": 150.0, "CORN": 230.0, "SUGAR_BEETS": 260.0},
}


def farmer_yields(scennum, crops_multiplier=1, seedoffset=0):
    """Yields of one farmer scenario, CROPS insertion order (farmer.py:159-183)."""
    base = _FARMER_BASE[scennum % 3]
    group = scennum // 3
    rs = np.random.RandomState()
    rs.seed(scennum + seedoffset)
    out = []
    for i in range(crops_multiplier):
        for crop in ["WHEAT", "CORN", "SUGAR_BEETS"]:
            y = _FARMER_YIELD[base][crop]
            if group != 0:
                y = y + rs.rand()
            out.append(y)
    return out


def farmer(sname, crops_multiplier=1, num_scens=None, seedoffset=0):
    scennum = extract_num(sname)
    cm = crops_multiplier
    crops = []
    for i in range(cm):
        crops += ["WHEAT%d" % i, "CORN%d" % i, "SUGAR_BEETS%d" % i]
    ylds = farmer_yields(scennum, cm, seedoffset)
    nc = len(crops)
    base = [re.sub(r"\d+$", "", c) for c in crops]
    # variable families: DA, QSub, QSuper, QP
    names = ["DevotedAcreage[%s]" % c for c in crops]
    names += ["QuantitySubQuotaSold[%s]" % c for c in crops]
    names += ["QuantitySuperQuotaSold[%s]" % c for c in crops]
    names += ["QuantityPurchased[%s]" % c for c in crops]
    n = 4 * nc
    DA, SUB, SUP, PUR = 0, nc, 2 * nc, 3 * nc
    c = np.zeros(n)
    lb = np.zeros(n)
    ub = np.full(n, INF)
    for k, b in enumerate(base):
        c[DA + k] = _FARMER_DATA["PlantingCostPerAcre"][b]
        c[PUR + k] = _FARMER_DATA["PurchasePrice"][b]
        c[SUB + k] = -_FARMER_DATA["SubQuotaSellingPrice"][b]
        c[SUP + k] = -_FARMER_DATA["SuperQuotaSellingPrice"][b]
        ub[DA + k] = 500.0 * cm
        ub[SUB + k] = _FARMER_DATA["PriceQuota"][b]  # EnforceQuotas folded to a bound
    rows, bl, bu = [], [], []
    r = np.zeros(n); r[DA:DA + nc] = 1.0
    rows.append(r); bl.append(-INF); bu.append(500.0 * cm)
    for k, b in enumerate(base):
        r = np.zeros(n)
        r[DA + k] = ylds[k]; r[PUR + k] = 1.0; r[SUB + k] = -1.0; r[SUP + k] = -1.0
        rows.append(r); bl.append(_FARMER_DATA["CattleFeedRequirement"][b]); bu.append(INF)
    for k, b in enumerate(base):
        r = np.zeros(n)
        r[SUB + k] = 1.0; r[SUP + k] = 1.0; r[DA + k] = -ylds[k]
        rows.append(r); bl.append(-INF); bu.append(0.0)
    nonant = sorted(range(nc), key=lambda k: crops[k])  # sorted(v.keys()): string sort
    prob = 1.0 / num_scens if num_scens is not None else None
    return Scen(sname, names, c, 0.0, np.array(rows), bl, bu, lb, ub,
                [("ROOT", 1.0, 1, [DA + k for k in nonant])], prob)


def docs_farmer(sname):
    """doc/src/examples.rst:56-94 + 175-190 (X[BEETS], X[CORN], X[WHEAT] sorted)."""
    yields = {"good": [3, 3.6, 24], "average": [2.5, 3, 20], "bad": [2, 2.4, 16]}[sname]
    # vars: X[W], X[C], X[B], Y[W], Y[C], W[W], W[C], W[BF], W[BU]
    names = ["X[WHEAT]", "X[CORN]", "X[BEETS]", "Y[WHEAT]", "Y[CORN]",
             "W[WHEAT]", "W[CORN]", "W[BEETS_FAVORABLE]", "W[BEETS_UNFAVORABLE]"]
    c = np.array([150, 230, 260, 238, 210, -170, -150, -36, -10], dtype=np.float64)
    lb = np.zeros(9)
    ub = np.full(9, INF); ub[7] = 6000.0
    A = np.zeros((4, 9))
    A[0, 0:3] = 1
    A[1, 0] = yields[0]; A[1, 3] = 1; A[1, 5] = -1
    A[2, 1] = yields[1]; A[2, 4] = 1; A[2, 6] = -1
    A[3, 2] = yields[2]; A[3, 7] = -1; A[3, 8] = -1
    bl = [-INF, 200, 240, 0]
    bu = [500, INF, INF, INF]
    return Scen(sname, names, c, 0.0, A, bl, bu, lb, ub,
                [("ROOT", 1.0, 1, [2, 1, 0])], 1.0 / 3)


# ---------------------------------------------------------------- aircond
AIRCOND_PARMS = {"mu_dev": 0.0, "sigma_dev": 40.0, "start_seed": 1134, "min_d": 0.0,
                 "max_d": 400.0, "starting_d": 200.0, "BeginInventory": 200.0,
                 "InventoryCost": 0.5, "LastInventoryCost": -0.8, "Capacity": 200.0,
                 "RegularProdCost": 1.0, "OvertimeProdCost": 3.0, "NegInventoryCost": 5.0}


def node_idx(node_path, branching_factors):
    """``sputils.node_idx`` (``utils/sputils.py:492-519``)."""
    if node_path == []:
        return 0
    stage_id = 0
    for t in range(len(node_path)):
        stage_id = node_path[t] + branching_factors[t] * stage_id
    before = int(sum(np.prod(branching_factors[0:i]) for i in range(len(node_path))))
    return before + stage_id


def aircond_demands(sname, branching_factors, **kw):
    """``aircond._demands_creator`` (``tests/examples/aircond.py:37-67``)."""
    p = dict(AIRCOND_PARMS); p.update(kw)
    scennum = extract_num(sname)
    prod = int(np.prod(branching_factors))
    s = int(scennum % prod)
    d = p["starting_d"]
    demands = [d]
    nodenames = ["ROOT"]
    for bf in branching_factors:
        prod = prod // bf
        nodenames.append(str(s // prod))
        s = s % prod
    stagelist = [int(x) for x in nodenames[1:]]
    rs = np.random.RandomState()
    for t in range(1, len(nodenames)):
        rs.seed(p["start_seed"] + node_idx(stagelist[:t], branching_factors))
        d = min(p["max_d"], max(p["min_d"], d + rs.normal(p["mu_dev"], p["sigma_dev"])))
        demands.append(d)
    return demands, nodenames


def aircond(sname, branching_factors, **kw):
    """aircond scenario (``aircond.py:88-301``), start_ups=False, QuadShortCoeff=0."""
    p = dict(AIRCOND_PARMS); p.update(kw)
    demands, nodenames = aircond_demands(sname, branching_factors, **kw)
    T = len(demands)
    bigM = p["Capacity"] * 25
    # per stage vars: RP, OP, Inv, neg, pos
    nv = 5
    n = nv * T
    names, c = [], np.zeros(n)
    lb, ub = np.zeros(n), np.zeros(n)
    for t in range(T):
        o = nv * t
        names += ["RegularProd[%d]" % (t + 1), "OvertimeProd[%d]" % (t + 1), "Inventory[%d]" % (t + 1),
                  "negInventory[%d]" % (t + 1), "posInventory[%d]" % (t + 1)]
        lb[o:o + 5] = [0, 0, -bigM, 0, 0]
        ub[o:o + 5] = [p["Capacity"], bigM, bigM, bigM, bigM]  # MaximumCapacity folded
        last = (t == T - 1)
        c[o + 0] = p["RegularProdCost"]
        c[o + 1] = p["OvertimeProdCost"]
        c[o + 3] = p["NegInventoryCost"]
        c[o + 4] = p["LastInventoryCost"] if last else p["InventoryCost"]
    rows, bl, bu = [], [], []
    for t in range(T):
        o = nv * t
        r = np.zeros(n)  # doleInventory: Inv - pos + neg == 0
        r[o + 2] = 1; r[o + 4] = -1; r[o + 3] = 1
        rows.append(r); bl.append(0.0); bu.append(0.0)
    for t in range(T):
        o = nv * t
        r = np.zeros(n)  # material balance
        r[o + 0] = 1; r[o + 1] = 1; r[o + 2] = -1
        rhs = demands[t]
        if t == 0:
            rhs = demands[t] - p["BeginInventory"]
        else:
            r[nv * (t - 1) + 2] = 1
        rows.append(r); bl.append(rhs); bu.append(rhs)
    nodes = []
    ndn = None
    for t in range(T - 1):
        o = nv * t
        if t == 0:
            ndn, cp = "ROOT", 1.0
        else:
            ndn, cp = ndn + "_" + nodenames[t], 1.0 / branching_factors[t - 1]
        nodes.append((ndn, cp, t + 1, [o + 0, o + 1]))
    prob = 1.0 / float(np.prod(branching_factors))
    return Scen(sname, names, c, 0.0, np.array(rows), bl, bu, lb, ub, nodes, prob)


def aircond_nodenames(branching_factors):
    """All non-leaf + leaf node names like ``sputils.create_nodenames_from_branching_factors``."""
    names = ["ROOT"]
    frontier = ["ROOT"]
    for bf in branching_factors:
        nxt = []
        for f in frontier:
            for b in range(bf):
                nxt.append("%s_%d" % (f, b))
        names += nxt
        frontier = nxt
    return names


# ---------------------------------------------------------------- sslp
_SSLP_JSON = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-sppy_amd", "examples",
                          "data", "sslp_15_45.json")


def sslp(sname, instance=None, num_scens=None):
    """sslp LP relaxation (``examples/sslp/model/ReferenceModel.py``): FacilityOpen,
    Allocation in [0,1], Dummy >= 0; demand rows sum_i D_ij A_ij - Dummy_j - Cap Open_j <= 0,
    client rows sum_j A_ij == ClientPresent_i.  Data from the reference's .dat files
    (extracted to sslp_15_45.json); unshipped scenarios draw ClientPresent ~
    Bernoulli(0.5) from RandomState(K)."""
    import json
    d = json.load(open(_SSLP_JSON))
    ns, nc = d["NumServers"], d["NumClients"]
    K = extract_num(sname)
    shipped = d["ClientPresent"].get(str(instance)) if instance is not None else None
    if shipped is not None and 1 <= K <= len(shipped):
        present = np.array(shipped[K - 1], dtype=np.float64)
    else:
        present = (np.random.RandomState(K).rand(nc) < 0.5).astype(np.float64)
    n = ns + nc * ns + ns
    names = ["FacilityOpen[%d]" % (j + 1) for j in range(ns)]
    names += ["Allocation[(%d, %d)]" % (i + 1, j + 1) for i in range(nc) for j in range(ns)]
    names += ["Dummy[%d]" % (j + 1) for j in range(ns)]
    c = np.zeros(n)
    lb = np.zeros(n)
    ub = np.ones(n)
    ub[ns + nc * ns:] = INF
    A = np.zeros((ns + nc, n))
    bl = np.zeros(ns + nc)
    bu = np.zeros(ns + nc)
    for j in range(ns):
        c[j] = d["FixedCost"][j]
        c[ns + nc * ns + j] = d["Penalty"]
        A[j, j] = -d["Capacity"]
        A[j, ns + nc * ns + j] = -1.0
        for i in range(nc):
            A[j, ns + i * ns + j] = d["Demand"][i][j]
        bl[j], bu[j] = -INF, 0.0
    for i in range(nc):
        for j in range(ns):
            c[ns + i * ns + j] = -d["Revenue"][i][j]
            A[ns + i, ns + i * ns + j] = 1.0
        bl[ns + i] = bu[ns + i] = present[i]
    prob = 1.0 / num_scens if num_scens is not None else None
    return Scen(sname, names, c, 0.0, A, bl, bu, lb, ub, [("ROOT", 1.0, 1, list(range(ns)))], prob)


# ---------------------------------------------------------------- netdes
def netdes(sname, instance="network-10-10-H-01", num_scens=None):
    """netdes LP relaxation (``examples/netdes/netdes.py:32-71``): x[e] in [0,1] then
    y[e] >= 0 per edge (edges = row-major nonzeros of the adjacency matrix,
    ``parse.py:58-59``); rows vubs y_e - u_e x_e <= 0, then bals (out-flow minus in-flow
    == b_i per node); cost c'x + d'y.  Data from the reference's .dat file (extracted to
    netdes_<instance>.npz); scenario index = trailing digits of the name (netdes.py:79-87);
    indices >= K take shipped scenario k mod K with d scaled by 1 + 0.2 (r - 1/2),
    r ~ RandomState(k).rand(E) (the build's synthetic workload)."""
    f = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-sppy_amd", "examples",
                     "data", "netdes_%s.npz" % instance)
    z = np.load(f)
    k = int(re.search(r"(\d+)$", sname).group(1))
    K = len(z["p"])
    ed = z["edges"]
    E, N = len(ed), int(z["N"])
    d, u, b = z["d"][k % K], z["u"][k % K], z["b"][k % K]
    if k >= K:
        d = d * (1.0 + 0.2 * (np.random.RandomState(k).rand(E) - 0.5))
    A = np.zeros((E + N, 2 * E))
    for e in range(E):
        A[e, e] = -u[e]
        A[e, E + e] = 1.0
        A[E + ed[e, 0], E + e] += 1.0
        A[E + ed[e, 1], E + e] -= 1.0
    bl = np.concatenate([np.full(E, -INF), b])
    bu = np.concatenate([np.zeros(E), b])
    names = ["x[%d,%d]" % (i, j) for i, j in ed] + ["y[%d,%d]" % (i, j) for i, j in ed]
    lb = np.zeros(2 * E)
    ub = np.concatenate([np.ones(E), np.full(E, INF)])
    prob = 1.0 / num_scens if num_scens is not None else (float(z["p"][k]) if k < K else None)
    return Scen(sname, names, np.concatenate([z["c"], d]), 0.0, A, bl, bu, lb, ub,
                [("ROOT", 1.0, 1, list(range(E)))], prob)


# ---------------------------------------------------------------- hydro
_HYDRO_JSON = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-sppy_amd", "examples",
                           "data", "hydro.json")


def hydro(sname, branching_factors=(3, 3)):
    """hydro / elec3 three-stage LP (``mpisppy/tests/examples/hydro/hydro.py:31-236``),
    written directly as a dense LP.  Columns: Pgt[1..3], Pgh[1..3], PDns[1..3],
    Vol[1..3], sl, StageCost[1..3].  Rows: StageCost[t] - r_t (bGt Pgt + bGh Pgh +
    bDns PDns) (- sl at t = 3) == 0; Pgt + Pgh + PDns == D[t]; Vol[t] - Vol[t-1] +
    u[t] Pgh[t] <= u[t] A[t] (Vol[0] = V0 on the right); sl + 4166.67 Vol[3] >=
    4166.67 V0.  r_t = (1/1.1)^(duracion[t]/T).  Nodes: ROOT [Pgt1, Pgh1, PDns1, Vol1],
    ROOT_<(snum-1)//bf0> (cond_prob 1/bf0) the same of stage 2; uniform probability."""
    import json
    p = json.load(open(_HYDRO_JSON))["scenarios"][sname]
    T = 3
    col = {}
    names = []
    for fam in ["Pgt", "Pgh", "PDns", "Vol"]:
        for t in range(1, T + 1):
            col[fam, t] = len(names)
            names.append("%s[%d]" % (fam, t))
    col["sl"] = len(names)
    names.append("sl")
    for t in range(1, T + 1):
        col["StageCost", t] = len(names)
        names.append("StageCost[%d]" % t)
    n = len(names)
    lb, ub = np.zeros(n), np.zeros(n)
    c = np.zeros(n)
    for t in range(1, T + 1):
        lb[col["Pgt", t]], ub[col["Pgt", t]] = p["PgtMin"], p["PgtMax"]
        lb[col["Pgh", t]], ub[col["Pgh", t]] = p["PghMin"], p["PghMax"]
        lb[col["PDns", t]], ub[col["PDns", t]] = 0.0, p["D"][str(t)]
        lb[col["Vol", t]], ub[col["Vol", t]] = p["VMin"], p["VMax"]
        lb[col["StageCost", t]], ub[col["StageCost", t]] = -INF, INF
        c[col["StageCost", t]] = 1.0
    lb[col["sl"]], ub[col["sl"]] = 0.0, INF
    rows, bl, bu = [], [], []
    for t in range(1, T + 1):
        r_t = (1.0 / 1.1) ** (p["duracion"][str(t)] / p["T"])
        a = np.zeros(n)
        a[col["StageCost", t]] = 1.0
        a[col["Pgt", t]] = -r_t * p["betaGt"]
        a[col["Pgh", t]] = -r_t * p["betaGh"]
        a[col["PDns", t]] = -r_t * p["betaDns"]
        if t == T:
            a[col["sl"]] = -1.0
        rows.append(a); bl.append(0.0); bu.append(0.0)
    for t in range(1, T + 1):
        a = np.zeros(n)
        a[col["Pgt", t]] = a[col["Pgh", t]] = a[col["PDns", t]] = 1.0
        rows.append(a); bl.append(p["D"][str(t)]); bu.append(p["D"][str(t)])
    for t in range(1, T + 1):
        a = np.zeros(n)
        u = p["u"][str(t)]
        a[col["Vol", t]] = 1.0
        a[col["Pgh", t]] = u
        rhs = u * p["A"][str(t)]
        if t == 1:
            rhs += p["V0"]
        else:
            a[col["Vol", t - 1]] = -1.0
        rows.append(a); bl.append(-INF); bu.append(rhs)
    a = np.zeros(n)
    a[col["sl"]] = 1.0
    a[col["Vol", T]] = 4166.67
    rows.append(a); bl.append(4166.67 * p["V0"]); bu.append(INF)
    snum = extract_num(sname)
    bf0 = branching_factors[0]
    nodes = [("ROOT", 1.0, 1, [col["Pgt", 1], col["Pgh", 1], col["PDns", 1], col["Vol", 1]]),
             ("ROOT_%d" % ((snum - 1) // bf0), 1.0 / bf0, 2,
              [col["Pgt", 2], col["Pgh", 2], col["PDns", 2], col["Vol", 2]])]
    return Scen(sname, names, c, 0.0, np.array(rows), bl, bu, lb, ub, nodes, None)
