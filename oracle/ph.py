"""Oracle PH loop — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Plain restatement of the reference hot path, ``PH.ph_main``
(``mpisppy/opt/ph.py:25-71``):

* ``Iter0``          phbase.py:758-872 — LP solve of every scenario with
                     W_on = prox_on = 0, trivial bound = sum_s p_s * obj_s
                     (``Ebound`` spopt.py:346-391).
* ``iterk_loop``     phbase.py:875-979 — per iteration:
                     ``Compute_Xbar`` (27-107, prob_coeff = p_s / uncond_prob(node),
                     spbase.py:378-391) -> ``Update_W`` (293-318,
                     W += rho (x - xbar)) -> ``convergence_diff`` (321-343: mean of
                     per-rank means of |x - xbar|) -> stop if conv < convthresh
                     (strict, before the solve) -> solve QPs with the PH terms of
                     ``attach_PH_to_objective`` (617-699).
* ``post_loops``     Eobjective (spopt.py:310-343) including W and prox terms.

Rank slicing for the conv normalisation follows ``_ScenTree.scen_names_to_ranks``
(``utils/sputils.py:803-810``): rank r owns range(int(r*S/R), int((r+1)*S/R)).
"""
import math
import numpy as np

from . import qp


def rank_slices(S, n_proc):
    if n_proc == 1:
        return [list(range(S))]
    avg = S / n_proc
    return [list(range(int(i * avg), int((i + 1) * avg))) for i in range(n_proc)]


class OraclePH:
    def __init__(self, scens, rho=1.0, n_proc=1, sense=1):
        self.scens = scens
        S = len(scens)
        for s in scens:
            if s.prob is None:
                s.prob = 1.0 / S
        self.S = S
        self.n_proc = n_proc
        self.sense = sense  # +1 min, -1 max (models here are min)
        # nonant slots: (node_name, i) in node-list order
        self.slots = []
        for (ndn, cp, st, vl) in scens[0].nodes:
            for i in range(len(vl)):
                self.slots.append((st, i))
        self.N = len(self.slots)
        # per-scenario nonant columns, node names per slot, prob_coeff per slot
        self.ncol = np.zeros((S, self.N), dtype=np.int64)
        self.node_of = [[None] * self.N for _ in range(S)]
        self.pc = np.zeros((S, self.N))
        for k, s in enumerate(scens):
            j = 0
            uncond = 1.0
            for (ndn, cp, st, vl) in s.nodes:
                uncond = uncond * cp if st > 1 else 1.0
                for v in vl:
                    self.ncol[k, j] = v
                    self.node_of[k][j] = ndn
                    self.pc[k, j] = s.prob / uncond
                    j += 1
        self.rho = np.full((S, self.N), float(rho))
        self.W = np.zeros((S, self.N))
        self.xbar = np.zeros((S, self.N))
        self.xsqbar = np.zeros((S, self.N))
        self.x = [None] * S
        self.obj = np.zeros(S)
        self.W_on = 0
        self.prox_on = 0
        self.conv = None
        self.iter = 0
        self.history = []

    # --- subproblem ---------------------------------------------------
    def _qp_data(self, k):
        s = self.scens[k]
        q = s.c.copy()
        p = np.zeros(len(q))
        cols = self.ncol[k]
        if self.W_on:
            q[cols] += self.W[k]
        if self.prox_on:
            q[cols] -= self.rho[k] * self.xbar[k]
            p[cols] += self.rho[k]
        return q, p

    def scen_objective(self, k, x):
        s = self.scens[k]
        f = float(np.dot(s.c, x)) + s.c0
        xn = x[self.ncol[k]]
        if self.W_on:
            f += float(np.dot(self.W[k], xn))
        if self.prox_on:
            f += float(np.sum(self.rho[k] / 2.0 * (xn * xn - 2.0 * self.xbar[k] * xn + self.xbar[k] ** 2)))
        return f

    def solve_loop(self):
        solve = getattr(self, "solver", None) or qp.solve
        for k, s in enumerate(self.scens):
            q, p = self._qp_data(k)
            x, feas = solve(s.A, s.bl, s.bu, s.lb, s.ub, q, p)
            if not feas:
                raise RuntimeError("oracle: infeasible scenario %s" % s.name)
            self.x[k] = x
            self.obj[k] = self.scen_objective(k, x)

    # --- PH pieces ----------------------------------------------------
    def xn(self):
        return np.array([self.x[k][self.ncol[k]] for k in range(self.S)])

    def compute_xbar(self):
        xn = self.xn()
        sums, sqs = {}, {}
        for k in range(self.S):
            for j in range(self.N):
                key = (self.node_of[k][j], j)
                sums[key] = sums.get(key, 0.0) + self.pc[k, j] * xn[k, j]
                sqs[key] = sqs.get(key, 0.0) + self.pc[k, j] * xn[k, j] ** 2
        for k in range(self.S):
            for j in range(self.N):
                key = (self.node_of[k][j], j)
                self.xbar[k, j] = sums[key]
                self.xsqbar[k, j] = sqs[key]

    def update_w(self):
        self.W += self.rho * (self.xn() - self.xbar)
        # variable probabilities: W of zero-probability nonants stays 0
        # (phbase.py:314-318, prob0_mask from spbase.py:394-434)
        if getattr(self, "prob0_mask", None) is not None:
            self.W *= self.prob0_mask

    def convergence_diff(self):
        xn = self.xn()
        tot = 0.0
        for sl in rank_slices(self.S, self.n_proc):
            d = 0.0
            cnt = 0
            for k in sl:
                d += float(np.sum(np.abs(xn[k] - self.xbar[k])))
                cnt += self.N
            tot += d / cnt
        return tot / self.n_proc

    def Ebound(self):
        return math.fsum(self.scens[k].prob * self.obj[k] for k in range(self.S))

    def Eobjective(self):
        return math.fsum(self.scens[k].prob * self.scen_objective(k, self.x[k]) for k in range(self.S))

    def iter0(self):
        self.iter = 0
        self.W_on = self.prox_on = 0
        self.solve_loop()
        self.trivial_bound = self.Ebound()
        self.W_on = self.prox_on = 1
        return self.trivial_bound

    def iterk(self, max_iterations, convthresh):
        self.conv = None
        for it in range(1, max_iterations + 1):
            self.iter = it
            self.compute_xbar()
            self.update_w()
            self.conv = self.convergence_diff()
            self.history.append(self.conv)
            if self.conv < convthresh:
                return it
            self.solve_loop()
        return max_iterations

    def ph_main(self, max_iterations, convthresh=1e-10):
        tb = self.iter0()
        self.iterk(max_iterations, convthresh)
        Eobj = self.Eobjective()
        return self.conv, Eobj, tb


def solve_ef(scens):
    """Extensive form (``sputils.create_EF``, utils/sputils.py:127-341) as one LP:
    scenario blocks plus nonanticipativity equalities x_s[slot] == x_ref(node)[slot]."""
    import scipy.sparse as sp
    S = len(scens)
    for s in scens:
        if s.prob is None:
            s.prob = 1.0 / S
    ns = [len(s.c) for s in scens]
    off = np.concatenate([[0], np.cumsum(ns)])
    n = int(off[-1])
    c = np.concatenate([s.prob * s.c for s in scens])
    lb = np.concatenate([s.lb for s in scens])
    ub = np.concatenate([s.ub for s in scens])
    blocks = [s.A for s in scens]
    A = sp.block_diag(blocks).toarray()
    bl = np.concatenate([s.bl for s in scens])
    bu = np.concatenate([s.bu for s in scens])
    first = {}
    extra = []
    for k, s in enumerate(scens):
        for (ndn, cp, st, vl) in s.nodes:
            for i, v in enumerate(vl):
                key = (ndn, i)
                if key not in first:
                    first[key] = off[k] + v
                else:
                    r = np.zeros(n)
                    r[off[k] + v] = 1.0
                    r[first[key]] = -1.0
                    extra.append(r)
    if extra:
        A = np.vstack([A, np.array(extra)])
        bl = np.concatenate([bl, np.zeros(len(extra))])
        bu = np.concatenate([bu, np.zeros(len(extra))])
    x, status = qp.highs_solve(A, bl, bu, lb, ub, c)
    obj = float(np.dot(c, x)) + sum(s.prob * s.c0 for s in scens)
    return obj, x, status


def evaluate_xhat(scens, cache, stage_max=None):
    """``Xhat_Eval.evaluate`` (utils/xhat_eval.py:297-327) restated: fix each
    scenario's nonants at ``cache[node][i]`` (lb = ub, spopt.py:557-591; only
    stages <= stage_max when given, xhat_eval.py:331-366), solve the LP and
    return (E[obj] = sum_s p_s obj_s, per-scenario objectives, feasible flags).
    Probabilities are the scenarios' own (a ``num_scens`` smaller than the name
    list makes them sum to more than 1, exactly as in the reference test)."""
    S = len(scens)
    objs = np.zeros(S)
    feas = np.zeros(S, dtype=bool)
    for k, s in enumerate(scens):
        if s.prob is None:
            s.prob = 1.0 / S
        lb, ub = s.lb.copy(), s.ub.copy()
        for (ndn, cp, st, vl) in s.nodes:
            if stage_max is not None and st > stage_max:
                continue
            vals = cache[ndn]
            for i, v in enumerate(vl):
                lb[v] = ub[v] = float(vals[i])
        x, ok = qp.solve(s.A, s.bl, s.bu, lb, ub, s.c, None)
        feas[k] = ok
        objs[k] = float(np.dot(s.c, x)) + s.c0 if ok else np.nan
    E = math.fsum(s.prob * o for s, o in zip(scens, objs))
    return E, objs, feas


def assign_bundles(S, n_proc, bundles_per_rank):
    """``SPBase._assign_bundles`` (spbase.py:219-253) restated: per rank, its
    contiguous scenario slice cut into bundles_per_rank slices range(int(i *
    avg), int((i + 1) * avg)), avg = count / bundles_per_rank."""
    out = []
    for sl in rank_slices(S, n_proc):
        avg = len(sl) / bundles_per_rank
        out += [[sl[i] for i in range(int(b * avg), int((b + 1) * avg))] for b in range(bundles_per_rank)]
    return out


class OracleBundledPH(OraclePH):
    """PH with EF bundles (``bundles_per_rank``): each bundle's subproblem is the
    extensive form of its scenarios as ``SPOpt.FormEF`` builds it
    (spopt.py:743-836, sputils.py:241-341): every scenario keeps its own
    variables, nonanticipativity equalities x_s[slot] == x_first[slot] per tree
    node, and the objective sum_s p_s (f_s + W_s x_s + rho/2 |x_s - xbar|^2) /
    p_bundle (normalised, sputils.py:273-275).  x-bar, W and the convergence
    metric stay per scenario (phbase.py:27-107, 293-343)."""

    def __init__(self, scens, bundles, rho=1.0, n_proc=1, sense=1):
        super().__init__(scens, rho=rho, n_proc=n_proc, sense=sense)
        self.bundles = [list(b) for b in bundles]

    def _bundle_qp(self, members):
        import scipy.sparse as sp
        pB = sum(self.scens[k].prob for k in members)
        qs, ps, As, bls, bus, lbs, ubs = [], [], [], [], [], [], []
        for k in members:
            q, p = self._qp_data(k)
            w = self.scens[k].prob / pB
            qs.append(w * q)
            ps.append(w * p)
            s = self.scens[k]
            As.append(s.A)
            bls.append(s.bl)
            bus.append(s.bu)
            lbs.append(s.lb)
            ubs.append(s.ub)
        ns = [len(self.scens[k].c) for k in members]
        off = np.concatenate([[0], np.cumsum(ns)])
        n = int(off[-1])
        A = sp.block_diag(As).toarray()
        bl, bu = np.concatenate(bls), np.concatenate(bus)
        first, extra = {}, []
        for b, k in enumerate(members):
            for j in range(self.N):
                key = (self.node_of[k][j], j)
                col = off[b] + self.ncol[k, j]
                if key not in first:
                    first[key] = col
                else:
                    r = np.zeros(n)
                    r[col], r[first[key]] = 1.0, -1.0
                    extra.append(r)
        if extra:
            A = np.vstack([A, np.array(extra)])
            bl = np.concatenate([bl, np.zeros(len(extra))])
            bu = np.concatenate([bu, np.zeros(len(extra))])
        return (A, bl, bu, np.concatenate(lbs), np.concatenate(ubs), np.concatenate(qs), np.concatenate(ps)), off

    def solve_loop(self):
        for members in self.bundles:
            (A, bl, bu, lb, ub, q, p), off = self._bundle_qp(members)
            x, feas = qp.solve(A, bl, bu, lb, ub, q, p)
            if not feas:
                raise RuntimeError("oracle: infeasible bundle %s" % members)
            for b, k in enumerate(members):
                self.x[k] = x[off[b]:off[b + 1]].copy()
                self.obj[k] = self.scen_objective(k, self.x[k])


def _prox_initial_points(lb, ub, count):
    """``ProxApproxManagerContinuous._create_initial_cuts`` (utils/prox_approx.py:124-141)."""
    pts = []
    if lb != 0.0:
        pts.append(float(lb))
    if lb == ub:
        return pts
    if ub != 0.0:
        pts.append(float(ub))
    if count > 2:
        delta = (ub - lb) / (count - 1)
        pts += [lb + i * delta for i in range(1, count - 1)]
    return pts


def _prox_newton(x_pnt, y_pnt):
    """``check_tol_add_cut``'s projection loop (utils/prox_approx.py:95-115)."""
    def step(v):
        return v - (v * (1 - 2 * y_pnt + 2 * v * v) - x_pnt) / (1 + 6 * v * v - 2 * y_pnt)
    this_val = x_pnt
    next_val = step(this_val)
    while not math.isclose(this_val, next_val, rel_tol=1e-6, abs_tol=1e-6):
        this_val = next_val
        next_val = step(this_val)
    return next_val


class OracleLinProxPH(OraclePH):
    """PH with ``linearize_proximal_terms`` (phbase.py:570-582, 617-699;
    utils/prox_approx.py): per scenario and nonant a variable xsq >= 0 with
    tangent cuts xsq >= 2 a x - a^2; the prox term is rho/2 (xsq - 2 xbar x +
    xbar^2), so prox-on subproblems are LPs.  Before each prox-on solve every
    nonant whose last (x, xsq) has x^2 - xsq > tol gets a cut at the Newton
    projection of that point onto y = x^2.  Prox-off solves are the plain LPs
    (xsq has zero cost there); xsq then takes its least feasible value
    max(0, max_k tangent_k(x)), the value of a simplex basis."""

    def __init__(self, scens, rho=1.0, tol=0.1, initial_cuts=2, n_proc=1, sense=1):
        super().__init__(scens, rho=rho, n_proc=n_proc, sense=sense)
        self.tol = tol
        self.cuts = []
        for k, s in enumerate(scens):
            row = []
            for j in range(self.N):
                col = self.ncol[k, j]
                lb, ub = float(s.lb[col]), float(s.ub[col])
                if not (math.isfinite(lb) and math.isfinite(ub)):
                    raise RuntimeError("linearize_nonbinary_proximal_terms requires bounded nonants")
                row.append(_prox_initial_points(lb, ub, initial_cuts))
            self.cuts.append(row)
        self.xsq = np.zeros((self.S, self.N))

    def _envelope(self, k, xn):
        return np.array([max([0.0] + [2 * a * xn[j] - a * a for a in self.cuts[k][j]]) for j in range(self.N)])

    def update_prox_approx(self):
        for k in range(self.S):
            xn = self.x[k][self.ncol[k]]
            for j in range(self.N):
                if xn[j] ** 2 - self.xsq[k, j] > self.tol:
                    self.cuts[k][j].append(_prox_newton(float(xn[j]), float(self.xsq[k, j])))

    def solve_loop(self):
        if not self.prox_on:
            super().solve_loop()
            for k in range(self.S):
                self.xsq[k] = self._envelope(k, self.x[k][self.ncol[k]])
            return
        if self.x[0] is not None:
            self.update_prox_approx()
        for k, s in enumerate(self.scens):
            n, N = len(s.c), self.N
            q = np.concatenate([s.c, 0.5 * self.rho[k]])
            cols = self.ncol[k]
            if self.W_on:
                q[cols] += self.W[k]
            q[cols] -= self.rho[k] * self.xbar[k]
            rows, bl, bu = [], [], []
            for j in range(N):
                for a in self.cuts[k][j]:
                    r = np.zeros(n + N)
                    r[cols[j]], r[n + j] = -2.0 * a, 1.0
                    rows.append(r)
                    bl.append(-a * a)
                    bu.append(np.inf)
            A = np.hstack([np.asarray(s.A.todense() if hasattr(s.A, "todense") else s.A), np.zeros((s.A.shape[0], N))])
            if rows:
                A = np.vstack([A, np.array(rows)])
            z, feas = qp.solve(A, np.concatenate([s.bl, bl]), np.concatenate([s.bu, bu]),
                               np.concatenate([s.lb, np.zeros(N)]), np.concatenate([s.ub, np.full(N, np.inf)]),
                               q, np.zeros(n + N))
            if not feas:
                raise RuntimeError("oracle: infeasible scenario %s" % s.name)
            self.x[k] = z[:n]
            self.xsq[k] = z[n:]
            self.obj[k] = self.scen_objective(k, self.x[k])

    def scen_objective(self, k, x):
        s = self.scens[k]
        f = float(np.dot(s.c, x)) + s.c0
        xn = x[self.ncol[k]]
        if self.W_on:
            f += float(np.dot(self.W[k], xn))
        if self.prox_on:
            xb = self.xbar[k]
            f += float(np.sum(self.rho[k] / 2.0 * (self.xsq[k] - 2.0 * xb * xn + xb ** 2)))
        return f
