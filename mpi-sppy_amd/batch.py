"""ScenarioBatch: the local scenarios in one shared-sparsity standard form.

Replaces what the reference holds as one Pyomo model + one solver plugin per
scenario (``SPBase._create_scenarios`` spbase.py:255-291,
``SPOpt._create_solvers`` spopt.py:839-903).  All local scenarios must share
one sparsity pattern; per-scenario numbers are stored scenario-minor
(``[i*S + s]``) and split into scenario-invariant and scenario-varying parts so
the device moves only the bytes that differ.

Two ways in, producing identical arrays (tested bit-exact):
  * ``from_models``: one ``LinearModel`` per scenario (the generic
    ``scenario_creator`` path of the reference API);
  * a vectorised ``batch_creator`` attached to a scenario creator
    (``scenario_creator.batch_creator(names, **kwargs) -> BatchData``), used
    for 10^5-scenario workloads.
"""
import numpy as np


class NonantSpec:
    """Scenario-tree / nonant description of the batch.

    slot_col[j]        column of nonant slot j (same for every scenario)
    slot_stage[j]      stage of the node owning slot j (1 = ROOT)
    slot_local[j]      index i of slot j inside its node, i.e. the ``i`` of the
                       reference's ``(ndn, i)`` nonant index (spbase.py:293-302)
    node_names[t]      for stage t (0-based over non-leaf stages): list of the
                       node name of every local scenario (None for 2-stage ROOT)
    cond_prob[t]       (S,) conditional probability of that node
    var_names          names of the nonant variables (for writers/views)
    """

    def __init__(self, slot_col, slot_stage, slot_local, node_names, cond_prob, var_names):
        self.slot_col = np.asarray(slot_col, dtype=np.int32)
        self.slot_stage = np.asarray(slot_stage, dtype=np.int32)
        self.slot_local = np.asarray(slot_local, dtype=np.int32)
        self.node_names = node_names
        self.cond_prob = cond_prob
        self.var_names = list(var_names)

    @property
    def N(self):
        return len(self.slot_col)

    @property
    def nstages(self):
        """number of non-leaf stages"""
        return int(self.slot_stage.max()) if self.N else 1

    def node_of(self, t, s):
        names = self.node_names[t]
        return "ROOT" if names is None else names[s]

    def nlen(self, t):
        return int(np.sum(self.slot_stage == t + 1))


class BatchData:
    """Host-side standard form of S local scenarios with a shared pattern.

    A-values: ``A_full`` (S, nnz) before compression; after ``compress()``:
    ``kvar`` (nnz,) with -1 for scenario-invariant entries, ``Aconst`` (nnz,),
    ``Avar`` (nvar, S).  Vectors c/lb/ub (n) and bl/bu (m) are either shared
    1-D arrays or (S, n|m) arrays (``*_vary`` flags).
    """

    def __init__(self, names, rowptr, colidx, A_full, bl, bu, lb, ub, c, c0, sense,
                 prob, nonant, var_names=None):
        self.names = list(names)
        self.S = len(self.names)
        self.rowptr = np.asarray(rowptr, dtype=np.int32)
        self.colidx = np.asarray(colidx, dtype=np.int32)
        self.m = len(self.rowptr) - 1
        self.nnz = int(self.rowptr[-1])
        self.A_full = np.asarray(A_full, dtype=np.float64).reshape(self.S, self.nnz)
        self.bl = np.asarray(bl, dtype=np.float64)
        self.bu = np.asarray(bu, dtype=np.float64)
        self.lb = np.asarray(lb, dtype=np.float64)
        self.ub = np.asarray(ub, dtype=np.float64)
        self.c = np.asarray(c, dtype=np.float64)
        self.n = self.c.shape[-1]
        self.c0 = np.broadcast_to(np.asarray(c0, dtype=np.float64), (self.S,)).copy()
        self.sense = sense
        self.prob = list(prob) if not isinstance(prob, np.ndarray) else prob
        self.nonant = nonant
        self.var_names = var_names
        self.kvar = None

    # ---------------------------------------------------------------
    @staticmethod
    def _squeeze(a, S):
        """(S, k) -> shared (k,) if every row equal, else keep (S, k)."""
        a = np.asarray(a, dtype=np.float64)
        if a.ndim == 1:
            return a, False
        if S == 1 or np.all(a == a[0:1]):
            return a[0].copy(), False
        return a, True

    def compress(self, force_var=None, force_rhs_vary=False):
        """Split invariant / varying parts (exact equality, NaN-free data).
        force_var: A entries kept varying even where equal now (a structure
        that must not change when they do); force_rhs_vary: row bounds per
        scenario."""
        S = self.S
        A = self.A_full
        same = np.all(A == A[0:1], axis=0) if S > 1 else np.ones(self.nnz, bool)
        if force_var is not None:
            same = same & ~np.asarray(force_var, dtype=bool)
        self.kvar = np.full(self.nnz, -1, dtype=np.int32)
        var_k = np.nonzero(~same)[0]
        self.kvar[var_k] = np.arange(len(var_k), dtype=np.int32)
        self.Aconst = np.where(same, A[0], 0.0).astype(np.float64)
        self.Avar = np.ascontiguousarray(A[:, var_k].T)          # (nvar, S)
        self.nvar = len(var_k)
        self.c, self.c_vary = self._squeeze(self.c, S)
        lb, lv = self._squeeze(self.lb, S)
        ub, uv = self._squeeze(self.ub, S)
        if lv or uv:
            self.lb = np.broadcast_to(self.lb, (S, self.n)).copy() if self.lb.ndim == 1 else self.lb
            self.ub = np.broadcast_to(self.ub, (S, self.n)).copy() if self.ub.ndim == 1 else self.ub
            self.bnd_vary = True
        else:
            self.lb, self.ub, self.bnd_vary = lb, ub, False
        bl, blv = self._squeeze(self.bl, S)
        bu, buv = self._squeeze(self.bu, S)
        if blv or buv or force_rhs_vary:
            self.bl = np.broadcast_to(self.bl, (S, self.m)).copy() if self.bl.ndim == 1 else self.bl
            self.bu = np.broadcast_to(self.bu, (S, self.m)).copy() if self.bu.ndim == 1 else self.bu
            self.rhs_vary = True
        else:
            self.bl, self.bu, self.rhs_vary = bl, bu, False
        return self

    # scenario-minor device layouts ------------------------------------
    def minor(self, a, vary):
        """(S, k) -> flat scenario-minor [k*S + s]; shared 1-D arrays unchanged."""
        return np.ascontiguousarray(a.T).ravel() if vary else np.ascontiguousarray(a)

    def scenario_A(self, s):
        """dense (m, n) matrix of local scenario s (tests / diagnostics)."""
        A = np.zeros((self.m, self.n))
        for i in range(self.m):
            for k in range(self.rowptr[i], self.rowptr[i + 1]):
                A[i, self.colidx[k]] = self.A_full[s, k] if self.kvar is None else (
                    self.Aconst[k] if self.kvar[k] < 0 else self.Avar[self.kvar[k], s])
        return A

    def vec(self, name, s):
        a = getattr(self, name)
        return a[s] if a.ndim == 2 else a


def from_models(names, models, sense=None):
    """Extract standard forms of per-scenario LinearModels into a BatchData."""
    S = len(models)
    sfs = [mdl.standard_form() for mdl in models]
    f0 = sfs[0]
    for k, f in enumerate(sfs):
        if len(f["c"]) != len(f0["c"]) or not np.array_equal(f["rowptr"], f0["rowptr"]) \
                or not np.array_equal(f["colidx"], f0["colidx"]):
            raise RuntimeError("scenario %s: sparsity pattern differs from scenario %s; the "
                               "batched engine needs one shared pattern" % (names[k], names[0]))
        if f["sense"] != f0["sense"]:
            raise RuntimeError("All scenario models must have the same model sense "
                               "(minimize or maximize)")
    A = np.stack([f["vals"] for f in sfs]) if f0["vals"].size else np.zeros((S, 0))
    nonant = nonant_spec_from_models(names, models)
    probs = [getattr(mdl, "_mpisppy_probability", None) for mdl in models]
    var_names = [v.name for v in models[0]._vars]
    return BatchData(names, f0["rowptr"], f0["colidx"], A,
                     np.stack([f["bl"] for f in sfs]), np.stack([f["bu"] for f in sfs]),
                     np.stack([f["lb"] for f in sfs]), np.stack([f["ub"] for f in sfs]),
                     np.stack([f["c"] for f in sfs]), np.array([f["c0"] for f in sfs]),
                     f0["sense"], probs, nonant, var_names)


def nonant_spec_from_models(names, models):
    m0 = models[0]
    if getattr(m0, "_mpisppy_node_list", None) is None:
        raise RuntimeError("_mpisppy_node_list not found on scenario %s" % names[0])
    slot_col, slot_stage, slot_local, vnames = [], [], [], []
    for node in m0._mpisppy_node_list:
        for i, v in enumerate(node.nonant_vardata_list):
            slot_col.append(v.index)
            slot_stage.append(node.stage)
            slot_local.append(i)
            vnames.append(v.name)
    T = max(slot_stage) if slot_stage else 1
    node_names = [None] * T
    cond_prob = [np.ones(len(models)) for _ in range(T)]
    for t in range(T):
        if t == 0:
            for k, mdl in enumerate(models):
                if mdl._mpisppy_node_list[0].name != "ROOT":
                    raise RuntimeError("first node of scenario %s must be ROOT" % names[k])
            continue
        node_names[t] = [mdl._mpisppy_node_list[t].name for mdl in models]
        cond_prob[t] = np.array([mdl._mpisppy_node_list[t].cond_prob for mdl in models], dtype=np.float64)
    for k, mdl in enumerate(models):
        cols = [v.index for node in mdl._mpisppy_node_list for v in node.nonant_vardata_list]
        if cols != slot_col:
            raise RuntimeError("scenario %s: nonant columns differ from scenario %s" % (names[k], names[0]))
    return NonantSpec(slot_col, slot_stage, slot_local, node_names, cond_prob, vnames)


def bundle_batch(b, groups, probs):
    """The EF bundles of a two-stage batch as one batch whose "scenarios" are
    the bundles (``SPOpt.subproblem_creation`` + ``FormEF``, spopt.py:743-836).

    groups[g]: local scenario indices of bundle g; probs: (S,) scenario
    probabilities.  Every bundle gets K = max group size member blocks (a
    smaller bundle repeats its first scenario with weight 0: the same rows on
    the same nonants, no cost -- the feasible nonants and the optimum are
    unchanged, and every bundle shares one sparsity pattern).  Column layout:
    [the N shared nonant columns | member 0's other columns | member 1's | ...];
    the nonant columns are shared (the EF's nonanticipativity equalities
    substituted out), their bounds the members' intersection.  Costs are
    weighted by p_s / p_bundle (the EF objective's normalisation,
    sputils.py:273-275), so the PH terms of the bundle lane are the weighted
    sums of its members' (SPOpt.solve_loop aggregates W and rho the same way).

    Returns (BatchData of the bundles, member index array (G, K), weights (G, K),
    column map (K, n): bundle column of each member column)."""
    nn = b.nonant
    if nn.nstages > 1:
        raise NotImplementedError("bundles of multistage trees (nonants below ROOT) are not supported")
    S, n, m, N = b.S, b.n, b.m, nn.N
    G = len(groups)
    K = max(len(g) for g in groups)
    members = np.array([list(g) + [g[0]] * (K - len(g)) for g in groups], dtype=np.int64)
    p = np.asarray(probs, dtype=np.float64)
    pB = np.array([sum(p[s] for s in g) for g in groups])
    wts = np.array([[p[s] / pB[gi] if r < len(g) else 0.0 for r, s in enumerate(members[gi])]
                    for gi, g in enumerate(groups)])
    slot_of = {int(c): t for t, c in enumerate(nn.slot_col)}
    others = [j for j in range(n) if j not in slot_of]
    no = len(others)
    colmap = np.zeros((K, n), dtype=np.int64)
    for r in range(K):
        for j in range(n):
            colmap[r, j] = slot_of[j] if j in slot_of else N + r * no + others.index(j)
    nB = N + K * no
    # rows: member r's rows, columns mapped and sorted within the row
    rowptr, colidx, src = [0], [], []          # src: (member, original nnz index) per bundle entry
    for r in range(K):
        for i in range(m):
            ks = list(range(b.rowptr[i], b.rowptr[i + 1]))
            ks.sort(key=lambda k: colmap[r, b.colidx[k]])
            for k in ks:
                colidx.append(int(colmap[r, b.colidx[k]]))
                src.append((r, k))
            rowptr.append(len(colidx))
    A = np.zeros((G, len(src)))
    for e, (r, k) in enumerate(src):
        A[:, e] = b.A_full[members[:, r], k]

    def per(a, width):
        a = np.asarray(a, dtype=np.float64)
        return a if a.ndim == 2 else np.broadcast_to(a, (S, width))

    c, lb, ub = per(b.c, n), per(b.lb, n), per(b.ub, n)
    bl, bu = per(b.bl, m), per(b.bu, m)
    cB = np.zeros((G, nB))
    lbB = np.zeros((G, nB))
    ubB = np.zeros((G, nB))
    lbB[:, :N], ubB[:, :N] = -np.inf, np.inf
    for r in range(K):
        sr = members[:, r]
        for j in range(n):
            q = colmap[r, j]
            cB[:, q] += wts[:, r] * c[sr, j]
            if q < N:
                lbB[:, q] = np.maximum(lbB[:, q], lb[sr, j])
                ubB[:, q] = np.minimum(ubB[:, q], ub[sr, j])
            else:
                lbB[:, q], ubB[:, q] = lb[sr, j], ub[sr, j]
    blB = np.concatenate([bl[members[:, r]] for r in range(K)], axis=1)
    buB = np.concatenate([bu[members[:, r]] for r in range(K)], axis=1)
    c0B = (wts * b.c0[members]).sum(axis=1)
    names = ["bundle%d" % g for g in range(G)]
    vn = [b.var_names[j] if b.var_names else "x%d" % j for j in nn.slot_col]
    spec = NonantSpec(np.arange(N), np.ones(N, dtype=np.int32), nn.slot_local, [None], [np.ones(G)], nn.var_names)
    out = BatchData(names, rowptr, colidx, A, blB, buB, lbB, ubB, cB, c0B, b.sense, pB, spec,
                    var_names=vn + ["b%d" % q for q in range(N, nB)])
    return out, members, wts, colmap
