"""Oracle subproblem solver — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Solves one scenario subproblem

    min  0.5 * x' diag(p) x + q' x + k
    s.t. bl <= A x <= bu,   lb <= x <= ub

the way the reference's ``SPOpt.solve_one`` (``mpisppy/spopt.py:85-223``)
does through an external solver: here scipy's bundled HiGHS 1.8.0 (LP simplex,
convex QP via ``passHessian``).  HiGHS's QP answer is only ~1e-5 accurate, so
the point is then *polished*: rows/bounds whose slack is tiny are taken as
active and the equality-constrained KKT system
``[[P, E'], [E, 0]] [x; lam] = [-q; e]`` is solved with least squares
(SURVEY.md §8(c) "Oracle recipe").  The polished point is accepted only when it
is primal feasible; otherwise the raw HiGHS point is returned.
"""
import numpy as np
from scipy.optimize._highspy import _core

INF = np.inf


def _to_highs_bound(v):
    v = np.asarray(v, dtype=np.float64).copy()
    v[v == INF] = _core.kHighsInf
    v[v == -INF] = -_core.kHighsInf
    return v


def highs_solve(A, bl, bu, lb, ub, q, p=None):
    """Solve with HiGHS. A dense (m, n). Returns (x, status_string)."""
    A = np.asarray(A, dtype=np.float64)
    m, n = A.shape
    h = _core._Highs()
    h.setOptionValue("output_flag", False)
    h.setOptionValue("primal_feasibility_tolerance", 1e-10)
    h.setOptionValue("dual_feasibility_tolerance", 1e-10)
    lp = _core.HighsLp()
    lp.num_col_ = n
    lp.num_row_ = m
    lp.col_cost_ = np.asarray(q, dtype=np.float64)
    lp.col_lower_ = _to_highs_bound(lb)
    lp.col_upper_ = _to_highs_bound(ub)
    lp.row_lower_ = _to_highs_bound(bl)
    lp.row_upper_ = _to_highs_bound(bu)
    # column-wise sparse matrix
    starts, idx, vals = [0], [], []
    for j in range(n):
        nzr = np.nonzero(A[:, j])[0]
        idx.extend(nzr.tolist())
        vals.extend(A[nzr, j].tolist())
        starts.append(len(idx))
    lp.a_matrix_.format_ = _core.MatrixFormat.kColwise
    lp.a_matrix_.start_ = np.asarray(starts, dtype=np.int32)
    lp.a_matrix_.index_ = np.asarray(idx, dtype=np.int32)
    lp.a_matrix_.value_ = np.asarray(vals, dtype=np.float64)
    lp.a_matrix_.num_col_ = n
    lp.a_matrix_.num_row_ = m
    h.passModel(lp)
    if p is not None and np.any(np.asarray(p) != 0):
        p = np.asarray(p, dtype=np.float64)
        hs = _core.HighsHessian()
        hs.dim_ = n
        hs.format_ = _core.HessianFormat.kTriangular
        nzc = np.nonzero(p)[0]
        st = np.zeros(n + 1, dtype=np.int32)
        for j in nzc:
            st[j + 1:] += 1
        hs.start_ = st
        hs.index_ = nzc.astype(np.int32)
        hs.value_ = p[nzc]
        h.passHessian(hs)
    h.run()
    status = h.modelStatusToString(h.getModelStatus())
    sol = h.getSolution()
    x = np.asarray(sol.col_value, dtype=np.float64)
    return x, status


def polish(A, bl, bu, lb, ub, q, p, x0, tol=1e-6):
    """Active-set KKT polish of an approximate optimum x0 (oracle recipe)."""
    A = np.asarray(A, dtype=np.float64)
    m, n = A.shape
    p = np.zeros(n) if p is None else np.asarray(p, dtype=np.float64)
    ax = A @ x0
    rows, rhs = [], []

    def near(a, b):
        return np.isfinite(b) and abs(a - b) <= tol * max(1.0, abs(b))

    for j in range(n):
        if near(x0[j], lb[j]):
            e = np.zeros(n); e[j] = 1.0; rows.append(e); rhs.append(lb[j])
        elif near(x0[j], ub[j]):
            e = np.zeros(n); e[j] = 1.0; rows.append(e); rhs.append(ub[j])
    for i in range(m):
        if near(ax[i], bl[i]):
            rows.append(A[i]); rhs.append(bl[i])
        elif near(ax[i], bu[i]):
            rows.append(A[i]); rhs.append(bu[i])
    E = np.array(rows).reshape(len(rows), n)
    k = E.shape[0]
    K = np.zeros((n + k, n + k))
    K[:n, :n] = np.diag(p)
    K[:n, n:] = E.T
    K[n:, :n] = E
    r = np.concatenate([-np.asarray(q, dtype=np.float64), np.asarray(rhs)])
    sol = np.linalg.lstsq(K, r, rcond=None)[0]
    return sol[:n]


def max_violation(A, bl, bu, lb, ub, x):
    ax = A @ x
    v = 0.0
    v = max(v, float(np.max(np.maximum(bl - ax, 0.0) / np.maximum(1.0, np.abs(np.where(np.isfinite(bl), bl, 0.0)))))) if len(ax) else v
    v = max(v, float(np.max(np.maximum(ax - bu, 0.0) / np.maximum(1.0, np.abs(np.where(np.isfinite(bu), bu, 0.0)))))) if len(ax) else v
    v = max(v, float(np.max(np.maximum(lb - x, 0.0))))
    v = max(v, float(np.max(np.maximum(x - ub, 0.0))))
    return v


def solve(A, bl, bu, lb, ub, q, p=None, do_polish=True):
    """HiGHS + polish.  Returns (x, feasible)."""
    x, status = highs_solve(A, bl, bu, lb, ub, q, p)
    if status != "Optimal":
        return x, False
    if not do_polish:
        return x, True
    xp = polish(A, bl, bu, lb, ub, q, p, x)
    if max_violation(A, bl, bu, lb, ub, xp) <= 1e-9:
        pp = np.zeros(len(x)) if p is None else np.asarray(p)
        f_raw = 0.5 * np.dot(pp * x, x) + np.dot(q, x)
        f_pol = 0.5 * np.dot(pp * xp, xp) + np.dot(q, xp)
        if f_pol <= f_raw + 1e-9 * max(1.0, abs(f_raw)):
            return xp, True
    return x, True
