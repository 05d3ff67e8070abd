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

    def compress(self):
        """Split invariant / varying parts (exact equality, NaN-free data)."""
        S = self.S
        A = self.A_full
        same = np.all(A == A[0:1], axis=0) if S > 1 else np.ones(self.nnz, bool)
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
        if blv or buv:
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
