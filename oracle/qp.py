"""Oracle subproblem solver — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Solves one scenario subproblem

    min  0.5 * x' diag(p) x + q' x + k
    s.t. bl <= A x <= bu,   lb <= x <= ub

the way the reference's ``SPOpt.solve_one`` (``mpisppy/spopt.py:85-223``)
does through an external solver: here scipy's bundled HiGHS 1.8.0 (LP simplex,
convex QP via ``passHessian``).  HiGHS's QP answer is only ~1e-5 accurate, so
the point is then *polished* (SURVEY.md §8(c) "Oracle recipe") and
*certified*:

1. the active set is read off HiGHS's basis (nonbasic columns / rows at their
   lower or upper bound), or off the point itself when there is no basis;
2. the equality-constrained KKT system of that active set
       P_FF x_F + q_F - A_RF' y_R = 0,   A_RF x_F = b_R - A_RB x_B
   is solved with a sparse LU (SuperLU); when it is singular (degenerate active
   sets), with a quasi-definite regularisation and iterative refinement on the
   unregularised system;
3. the point passes a KKT certificate — primal feasibility of every row and
   bound, correctly signed multipliers of every active row / bound and the
   stationarity residual, all relative 1e-9 — or the active set is updated
   (wrong-signed multipliers leave, violated constraints enter, the
   primal-dual active-set rule) and step 2 repeats.

A point that never certifies raises ``Uncertified`` (no silent fallback to the
raw HiGHS point).  Matrices may be dense or scipy.sparse.
"""
import numpy as np
import scipy.sparse as sps
import scipy.sparse.linalg as spla
from scipy.optimize._highspy import _core

INF = np.inf
_BS = _core.HighsBasisStatus


class Uncertified(RuntimeError):
    """The polished point failed the KKT certificate within the round budget."""


def _to_highs_bound(v):
    v = np.asarray(v, dtype=np.float64).copy()
    v[v == INF] = _core.kHighsInf
    v[v == -INF] = -_core.kHighsInf
    return v


def as_csc(A):
    return A.tocsc() if sps.issparse(A) else sps.csc_matrix(np.asarray(A, dtype=np.float64))


def highs_solve(A, bl, bu, lb, ub, q, p=None, want_basis=False):
    """Solve with HiGHS.  Returns (x, status_string) or, with want_basis,
    (x, status_string, col_status, row_status) (HighsBasisStatus ints, or None)."""
    Ac = as_csc(A)
    m, n = Ac.shape
    h = _core._Highs()
    h.setOptionValue("output_flag", False)
    h.setOptionValue("primal_feasibility_tolerance", 1e-10)
    h.setOptionValue("dual_feasibility_tolerance", 1e-10)
    # HiGHS 1.8's active-set QP solver can cycle (sslp prox QPs): bounded, the
    # caller then falls back to ipm_qp
    h.setOptionValue("qp_iteration_limit", 20000)
    h.setOptionValue("time_limit", 20.0)
    lp = _core.HighsLp()
    lp.num_col_ = n
    lp.num_row_ = m
    lp.col_cost_ = np.asarray(q, dtype=np.float64)
    lp.col_lower_ = _to_highs_bound(lb)
    lp.col_upper_ = _to_highs_bound(ub)
    lp.row_lower_ = _to_highs_bound(bl)
    lp.row_upper_ = _to_highs_bound(bu)
    lp.a_matrix_.format_ = _core.MatrixFormat.kColwise
    lp.a_matrix_.start_ = Ac.indptr.astype(np.int32)
    lp.a_matrix_.index_ = Ac.indices.astype(np.int32)
    lp.a_matrix_.value_ = Ac.data.astype(np.float64)
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
        st[1:] = np.cumsum(p != 0)
        hs.start_ = st
        hs.index_ = nzc.astype(np.int32)
        hs.value_ = p[nzc]
        h.passHessian(hs)
    h.run()
    status = h.modelStatusToString(h.getModelStatus())
    sol = h.getSolution()
    x = np.asarray(sol.col_value, dtype=np.float64)
    if not want_basis:
        return x, status
    cs = rs = None
    try:
        b = h.getBasis()
        if b.valid:
            cs = np.array([int(v) for v in b.col_status])
            rs = np.array([int(v) for v in b.row_status])
    except Exception:          # no basis from this solver path
        pass
    return x, status, cs, rs


def _initial_active_set(Ar, bl, bu, lb, ub, x0, cs, rs, tol=1e-7, lam=None, y0=None):
    """Column codes (0 free, 1 at lb, 2 at ub) and row codes (0 inactive, 1 at bl,
    2 at bu) from HiGHS's basis; else from the point: near a finite bound, or
    (with multipliers: lam = reduced costs, y0 = row multipliers) a slack smaller
    than its correctly signed multiplier (strict complementarity at an
    interior point)."""
    n, m = len(x0), len(bl)
    cc = np.zeros(n, dtype=np.int8)
    rc = np.zeros(m, dtype=np.int8)
    if cs is not None and rs is not None and len(cs) == n and len(rs) == m:
        lo, up = int(_BS.kLower), int(_BS.kUpper)
        cc[(cs == lo) & np.isfinite(lb)] = 1
        cc[(cs == up) & np.isfinite(ub)] = 2
        rc[(rs == lo) & np.isfinite(bl)] = 1
        rc[(rs == up) & np.isfinite(bu)] = 2
        return cc, rc
    ax = Ar @ x0
    near = lambda a, b: np.isfinite(b) & (np.abs(a - b) <= tol * np.maximum(1.0, np.abs(np.where(np.isfinite(b), b, 0.0))))
    fin = lambda v: np.where(np.isfinite(v), v, 0.0)
    at_l, at_u = near(x0, lb), near(x0, ub)
    at_bl, at_bu = near(ax, bl), near(ax, bu)
    if lam is not None:
        at_l |= np.isfinite(lb) & (x0 - fin(lb) < lam)
        at_u |= np.isfinite(ub) & (fin(ub) - x0 < -lam)
    if y0 is not None:
        at_bl |= np.isfinite(bl) & (ax - fin(bl) < y0)
        at_bu |= np.isfinite(bu) & (fin(bu) - ax < -y0)
    cc[at_l] = 1
    cc[(cc == 0) & at_u] = 2
    rc[at_bl] = 1
    rc[(rc == 0) & at_bu] = 2
    return cc, rc


def _kkt_solve(Ac, Ar, p, q, bl, bu, lb, ub, cc, rc, x_seed, y_seed):
    """Solve the KKT system of the active set (cc, rc).  Returns (x, y) with y the
    row multipliers (0 on inactive rows); None if the system is inconsistent."""
    n, m = Ac.shape[1], Ar.shape[0]
    F = np.nonzero(cc == 0)[0]
    B = np.nonzero(cc != 0)[0]
    R = np.nonzero(rc != 0)[0]
    x = x_seed.copy()
    x[cc == 1] = lb[cc == 1]
    x[cc == 2] = ub[cc == 2]
    bR = np.where(rc[R] == 1, bl[R], bu[R])
    A_R = Ar[R]
    A_RF = A_R[:, F]
    rhs2 = bR - A_R[:, B] @ x[B]
    nF, nR = len(F), len(R)
    K = sps.bmat([[sps.diags(p[F]), -A_RF.T], [A_RF, None]], format="csc") if nR else sps.diags(p[F]).tocsc()
    r = np.concatenate([-q[F], rhs2])
    sol = None
    if nF + nR == 0:
        sol = np.zeros(0)
    else:
        try:
            lu = spla.splu(K)
            s = lu.solve(r)
            if np.all(np.isfinite(s)):
                for _ in range(3):          # refinement of the exact factor
                    s = s + lu.solve(r - K @ s)
                sol = s
        except RuntimeError:                # exactly singular (degenerate active set)
            sol = None
        if sol is None or not np.all(np.isfinite(sol)) or \
                np.max(np.abs(K @ sol - r)) > 1e-9 * (1.0 + np.max(np.abs(r))):
            # quasi-definite regularisation + proximal-point refinement on K
            scale = 1.0 + (abs(K).max() if K.nnz else 0.0)
            d = 1e-8 * scale
            Kr = (K + sps.diags(np.concatenate([np.full(nF, d), np.full(nR, -d)]))).tocsc()
            lu = spla.splu(Kr)
            s = np.concatenate([x_seed[F], y_seed[R] if y_seed is not None else np.zeros(nR)])
            for _ in range(200):
                ds = lu.solve(r - K @ s)
                s = s + ds
                if np.max(np.abs(ds)) <= 1e-13 * (1.0 + np.max(np.abs(s))):
                    break
            sol = s
    x[F] = sol[:nF]
    y = np.zeros(m)
    y[R] = sol[nF:]
    return x, y


def certified_polish(A, bl, bu, lb, ub, q, p, x0, cs=None, rs=None, y0=None, tol=1e-9, max_rounds=60):
    """Active-set KKT polish of an approximate optimum x0 with a KKT certificate.
    Returns (x, y, rounds); raises Uncertified when no round certifies."""
    Ac = as_csc(A)
    Ar = Ac.tocsr()
    n, m = Ac.shape[1], Ac.shape[0]
    q = np.asarray(q, dtype=np.float64)
    p = np.zeros(n) if p is None else np.asarray(p, dtype=np.float64)
    bl, bu = np.asarray(bl, dtype=np.float64), np.asarray(bu, dtype=np.float64)
    lb, ub = np.asarray(lb, dtype=np.float64), np.asarray(ub, dtype=np.float64)
    lam = None if y0 is None else p * x0 + q - Ac.T @ np.asarray(y0, dtype=np.float64)
    cc, rc = _initial_active_set(Ar, bl, bu, lb, ub, x0, cs, rs, lam=lam, y0=y0)
    dtol = tol * (1.0 + np.max(np.abs(q))) if n else tol
    fin = lambda v: np.where(np.isfinite(v), v, 0.0)
    x, y = x0.copy(), (np.zeros(m) if y0 is None else np.asarray(y0, dtype=np.float64).copy())
    for rnd in range(1, max_rounds + 1):
        x, y = _kkt_solve(Ac, Ar, p, q, bl, bu, lb, ub, cc, rc, x, y)
        ax = Ar @ x
        z = p * x + q - Ac.T @ y                      # bound multipliers (stationarity of F: ~0)
        vb_lo = (lb - x) > tol * (1.0 + np.abs(fin(lb)))
        vb_up = (x - ub) > tol * (1.0 + np.abs(fin(ub)))
        vr_lo = (bl - ax) > tol * (1.0 + np.abs(fin(bl)))
        vr_up = (ax - bu) > tol * (1.0 + np.abs(fin(bu)))
        fixed = lb == ub
        eqr = bl == bu
        wz_lo = (cc == 1) & ~fixed & (z < -dtol)
        wz_up = (cc == 2) & ~fixed & (z > dtol)
        wy_lo = (rc == 1) & ~eqr & (y < -dtol)
        wy_up = (rc == 2) & ~eqr & (y > dtol)
        stat = (cc == 0) & (np.abs(z) > dtol)
        if not (vb_lo.any() or vb_up.any() or vr_lo.any() or vr_up.any() or wz_lo.any() or wz_up.any()
                or wy_lo.any() or wy_up.any() or stat.any()):
            return x, y, rnd
        # primal-dual active-set update
        cc[wz_lo | wz_up] = 0
        cc[(cc == 0) & vb_lo] = 1
        cc[(cc == 0) & vb_up] = 2
        rc[wy_lo | wy_up] = 0
        y[wy_lo | wy_up] = 0.0
        rc[(rc == 0) & vr_lo] = 1
        rc[(rc == 0) & vr_up] = 2
    raise Uncertified("KKT certificate not reached in %d active-set rounds" % max_rounds)


def max_violation(A, bl, bu, lb, ub, x):
    ax = as_csc(A) @ x
    v = 0.0
    v = max(v, float(np.max(np.maximum(bl - ax, 0.0) / np.maximum(1.0, np.abs(np.where(np.isfinite(bl), bl, 0.0)))))) if len(ax) else v
    v = max(v, float(np.max(np.maximum(ax - bu, 0.0) / np.maximum(1.0, np.abs(np.where(np.isfinite(bu), bu, 0.0)))))) if len(ax) else v
    v = max(v, float(np.max(np.maximum(lb - x, 0.0))))
    v = max(v, float(np.max(np.maximum(x - ub, 0.0))))
    return v


def ipm_qp(A, bl, bu, lb, ub, q, p, tol=1e-10, max_it=100):
    """Primal-dual Mehrotra interior point for the convex QP, written
    independently of the engine's (augmented system [[P + Dx, -A'], [A, Dr]]
    factored by SuperLU, not normal equations).  For QPs too large for HiGHS's
    active-set QP solver in reasonable time (netdes-50-30-H: n = 2,940).
    Returns (x, y, feasible) with y the row multipliers (y > 0: lower side)."""
    Ac = as_csc(A)
    Ar = Ac.tocsr()
    m, n = Ar.shape
    q = np.asarray(q, dtype=np.float64)
    p = np.zeros(n) if p is None else np.asarray(p, dtype=np.float64)
    fl, fu = np.isfinite(lb), np.isfinite(ub)
    fix = fl & fu & (lb == ub)
    fl &= ~fix
    fu &= ~fix
    eq = np.isfinite(bl) & np.isfinite(bu) & (bl == bu)
    rl, ru = np.isfinite(bl) & ~eq, np.isfinite(bu) & ~eq
    free_row = ~eq & ~rl & ~ru
    L = np.where(fl, lb, 0.0); U = np.where(fu, ub, 0.0)
    BL = np.where(rl, bl, 0.0); BU = np.where(ru, bu, 0.0)
    x = np.where(fix, np.where(np.isfinite(lb), lb, 0.0), 0.0)
    both = fl & fu
    x = np.where(both, 0.5 * (L + U), x)
    x = np.where(fl & ~fu, L + 1.0, x)
    x = np.where(fu & ~fl, U - 1.0, x)
    s = Ar @ x
    s = np.where(rl & ru, 0.5 * (BL + BU), s)
    s = np.where(rl & ~ru, np.maximum(s, BL + 1.0), s)
    s = np.where(ru & ~rl, np.minimum(s, BU - 1.0), s)
    g = q + p * x                        # cost-aware start: bound multipliers absorb the cost
    zl = np.where(fl, np.maximum(g, 0.0) + 1.0, 0.0); zu = np.where(fu, np.maximum(-g, 0.0) + 1.0, 0.0)
    wl = np.where(rl, 1.0, 0.0); wu = np.where(ru, 1.0, 0.0)
    y = wl - wu
    nc = int(fl.sum() + fu.sum() + rl.sum() + ru.sum())
    scale_q = 1.0 + np.max(np.abs(q))
    scale_b = 1.0 + max(np.max(np.abs(np.where(np.isfinite(bl), bl, 0.0)), initial=0.0),
                        np.max(np.abs(np.where(np.isfinite(bu), bu, 0.0)), initial=0.0))
    inv = lambda v, msk: np.where(msk, 1.0 / np.where(msk, v, 1.0), 0.0)
    # Newton matrix couplings: free rows (y = 0) and fixed columns (dx = 0) drop out
    Au = (sps.diags((~free_row).astype(np.float64)) @ Ar @ sps.diags((~fix).astype(np.float64))).tocsr()
    for it in range(max_it):
        gl, gu = np.where(fl, x - L, 1.0), np.where(fu, U - x, 1.0)
        hl, hu = np.where(rl, s - BL, 1.0), np.where(ru, BU - s, 1.0)
        rd = p * x + q - Ac.T @ y - zl + zu
        rd[fix] = 0.0
        ax = Ar @ x
        rp = np.where(eq, ax - np.where(eq, bl, 0.0), ax - s)
        rp[free_row] = 0.0
        ry = np.where(eq | free_row, 0.0, y - wl + wu)
        mu = (np.sum(np.where(fl, gl * zl, 0)) + np.sum(np.where(fu, gu * zu, 0)) +
              np.sum(np.where(rl, hl * wl, 0)) + np.sum(np.where(ru, hu * wu, 0))) / max(nc, 1)
        err = max(np.max(np.abs(rd), initial=0.0) / scale_q, np.max(np.abs(rp), initial=0.0) / scale_b,
                  np.max(np.abs(ry), initial=0.0) / scale_q, mu / (scale_q * scale_b))
        if err < tol:
            break
        Dx = np.where(fl, zl / gl, 0.0) + np.where(fu, zu / gu, 0.0) + p
        Dx = np.where(fix, 1.0, Dx + 1e-12)
        Ds = np.where(rl, wl / hl, 0.0) + np.where(ru, wu / hu, 0.0)
        Dr = np.where(eq, 1e-12, np.where(free_row, 1.0, inv(Ds, ~eq & ~free_row)))
        K = sps.bmat([[sps.diags(Dx), -Au.T], [Au, sps.diags(Dr)]], format="csc")
        lu = spla.splu(K)

        def direction(cl, cu, cwl, cwu):
            # complementarity targets: (x-L)dzl + zl dx = cl - (x-L)zl ... folded into rhs
            r1 = -rd + np.where(fl, cl / gl, 0.0) - np.where(fu, cu / gu, 0.0)
            r1[fix] = 0.0
            # inequality rows: ds = (dy + ry - rhs_w) / Ds ; A dx - ds = -rp
            rw = np.where(rl, cwl / hl, 0.0) - np.where(ru, cwu / hu, 0.0)
            r2 = np.where(eq, -rp, np.where(free_row, 0.0, -rp + inv(Ds, ~eq & ~free_row) * (-ry + rw)))
            sol = lu.solve(np.concatenate([r1, r2]))
            dx, dy = sol[:n], sol[n:]
            dx[fix] = 0.0
            ds = np.where(eq | free_row, 0.0, inv(Ds, ~eq & ~free_row) * (rw - ry - dy))
            dzl = np.where(fl, (cl - zl * dx) / gl, 0.0)
            dzu = np.where(fu, (cu + zu * dx) / gu, 0.0)
            dwl = np.where(rl, (cwl - wl * ds) / hl, 0.0)
            dwu = np.where(ru, (cwu + wu * ds) / hu, 0.0)
            return dx, dy, ds, dzl, dzu, dwl, dwu

        def steps(dx, ds, dzl, dzu, dwl, dwu):
            def mx(v, d, msk):
                k = msk & (d < 0)
                return float(np.min(-v[k] / d[k])) if k.any() else 1.0
            ap = min(1.0, mx(gl, dx, fl), mx(gu, -dx, fu), mx(hl, ds, rl), mx(hu, -ds, ru))
            ad = min(1.0, mx(zl, dzl, fl), mx(zu, dzu, fu), mx(wl, dwl, rl), mx(wu, dwu, ru))
            return ap, ad

        d = direction(-gl * zl, -gu * zu, -hl * wl, -hu * wu)
        ap, ad = steps(d[0], d[2], d[3], d[4], d[5], d[6])
        maff = (np.sum(np.where(fl, (gl + ap * d[0]) * (zl + ad * d[3]), 0)) +
                np.sum(np.where(fu, (gu - ap * d[0]) * (zu + ad * d[4]), 0)) +
                np.sum(np.where(rl, (hl + ap * d[2]) * (wl + ad * d[5]), 0)) +
                np.sum(np.where(ru, (hu - ap * d[2]) * (wu + ad * d[6]), 0))) / max(nc, 1)
        smu = min(1.0, maff / mu) ** 3 * mu if mu > 0 else 0.0
        d = direction(smu - gl * zl - d[0] * d[3], smu - gu * zu + d[0] * d[4],
                      smu - hl * wl - d[2] * d[5], smu - hu * wu + d[2] * d[6])
        ap, ad = steps(d[0], d[2], d[3], d[4], d[5], d[6])
        ap, ad = min(1.0, 0.995 * ap), min(1.0, 0.995 * ad)
        x = x + ap * d[0]; s = s + ap * d[2]; y = y + ad * d[1]
        zl = zl + ad * d[3]; zu = zu + ad * d[4]; wl = wl + ad * d[5]; wu = wu + ad * d[6]
    else:
        return x, y, False
    return x, y, True


STATS = {"solves": 0, "rounds": 0, "ipm": 0}
IPM_ABOVE = 1000      # QPs with more columns go through ipm_qp instead of HiGHS's QP solver


def solve(A, bl, bu, lb, ub, q, p=None, do_polish=True):
    """HiGHS (LP; QP up to IPM_ABOVE columns) or ipm_qp, then the certified
    polish.  Returns (x, feasible); raises Uncertified if a feasible problem's
    point cannot be certified."""
    n = np.shape(A)[1]
    if p is not None and np.any(np.asarray(p) != 0) and n > IPM_ABOVE:
        x, y, ok = ipm_qp(A, bl, bu, lb, ub, q, p)
        STATS["ipm"] += 1
        if not ok:
            return x, False
        if not do_polish:
            return x, True
        xp, _, rounds = certified_polish(A, bl, bu, lb, ub, q, p, x, y0=y)
    else:
        x, status, cs, rs = highs_solve(A, bl, bu, lb, ub, q, p, want_basis=True)
        is_qp = p is not None and np.any(np.asarray(p) != 0)
        if status != "Optimal" and is_qp and status in ("Iteration limit reached", "Time limit reached"):
            x, y, ok = ipm_qp(A, bl, bu, lb, ub, q, p)
            STATS["ipm"] += 1
            if not ok:
                return x, False
            xp, _, rounds = certified_polish(A, bl, bu, lb, ub, q, p, x, y0=y)
            STATS["solves"] += 1
            STATS["rounds"] += rounds
            return xp, True
        if status != "Optimal":
            return x, False
        if not do_polish:
            return x, True
        xp, _, rounds = certified_polish(A, bl, bu, lb, ub, q, p, x, cs, rs)
    STATS["solves"] += 1
    STATS["rounds"] += rounds
    return xp, True


def _certified(A, bl, bu, lb, ub, q, p, x, y, cc, rc, tol=1e-9):
    """certified_polish's KKT certificate of (x, y) for the active set (cc, rc), dense."""
    fin = lambda v: np.where(np.isfinite(v), v, 0.0)
    ax = A @ x
    z = p * x + q - A.T @ y
    dtol = tol * (1.0 + np.max(np.abs(q))) if len(q) else tol
    bad = ((lb - x) > tol * (1.0 + np.abs(fin(lb)))).any() or ((x - ub) > tol * (1.0 + np.abs(fin(ub)))).any()
    bad = bad or ((bl - ax) > tol * (1.0 + np.abs(fin(bl)))).any() or ((ax - bu) > tol * (1.0 + np.abs(fin(bu)))).any()
    fixed, eqr = lb == ub, bl == bu
    bad = bad or ((cc == 1) & ~fixed & (z < -dtol)).any() or ((cc == 2) & ~fixed & (z > dtol)).any()
    bad = bad or ((rc == 1) & ~eqr & (y < -dtol)).any() or ((rc == 2) & ~eqr & (y > dtol)).any()
    bad = bad or ((cc == 0) & (np.abs(z) > dtol)).any()
    return not bad


class PersistentHighs:
    """One HiGHS instance per subproblem, kept across PH iterations: each solve
    changes only the costs and the (diagonal) prox Hessian and re-runs from the
    previous basis -- the analogue of the reference's persistent solver plugins
    (``spopt.py:129-142``: set_instance once, set_objective per solve)."""

    def __init__(self, A, bl, bu, lb, ub):
        Ac = as_csc(A)
        m, n = Ac.shape
        self.n = n
        h = _core._Highs()
        h.setOptionValue("output_flag", False)
        h.setOptionValue("primal_feasibility_tolerance", 1e-10)
        h.setOptionValue("dual_feasibility_tolerance", 1e-10)
        h.setOptionValue("qp_iteration_limit", 20000)
        h.setOptionValue("time_limit", 20.0)
        lp = _core.HighsLp()
        lp.num_col_, lp.num_row_ = n, m
        lp.col_cost_ = np.zeros(n)
        lp.col_lower_, lp.col_upper_ = _to_highs_bound(lb), _to_highs_bound(ub)
        lp.row_lower_, lp.row_upper_ = _to_highs_bound(bl), _to_highs_bound(bu)
        lp.a_matrix_.format_ = _core.MatrixFormat.kColwise
        lp.a_matrix_.start_ = Ac.indptr.astype(np.int32)
        lp.a_matrix_.index_ = Ac.indices.astype(np.int32)
        lp.a_matrix_.value_ = Ac.data.astype(np.float64)
        lp.a_matrix_.num_col_, lp.a_matrix_.num_row_ = n, m
        h.passModel(lp)
        self.h = h
        self.cols = np.arange(n, dtype=np.int32)

    def solve(self, q, p):
        h, n = self.h, self.n
        h.changeColsCost(n, self.cols, np.asarray(q, dtype=np.float64))
        hs = _core.HighsHessian()
        hs.dim_ = n
        hs.format_ = _core.HessianFormat.kTriangular
        nzc = np.nonzero(p)[0]
        st = np.zeros(n + 1, dtype=np.int32)
        st[1:] = np.cumsum(p != 0)
        hs.start_, hs.index_, hs.value_ = st, nzc.astype(np.int32), p[nzc]
        h.passHessian(hs)
        h.run()
        status = h.modelStatusToString(h.getModelStatus())
        x = np.asarray(h.getSolution().col_value, dtype=np.float64)
        cs = rs = None
        b = h.getBasis()
        if b.valid:
            cs = np.array([int(v) for v in b.col_status])
            rs = np.array([int(v) for v in b.row_status])
        return x, status, cs, rs


def solve_fast(A, bl, bu, lb, ub, q, p=None, hs=None):
    """The CPU baseline's subproblem solve (oracle/cpu_bench.py): HiGHS (hs: the
    subproblem's PersistentHighs), then ONE dense KKT polish of HiGHS's basis; the
    iterated certified polish (solve) runs only when that point fails the same
    certificate.  Dense A (small subproblems: farmer).  Returns (x, feasible)."""
    n = A.shape[1]
    q = np.asarray(q, dtype=np.float64)
    p = np.zeros(n) if p is None else np.asarray(p, dtype=np.float64)
    if hs is not None:
        x0, status, cs, rs = hs.solve(q, p)
    else:
        x0, status, cs, rs = highs_solve(A, bl, bu, lb, ub, q, p, want_basis=True)
    if status != "Optimal" or cs is None:
        return solve(A, bl, bu, lb, ub, q, p)
    cc, rc = _initial_active_set(A, bl, bu, lb, ub, x0, cs, rs)
    F = np.nonzero(cc == 0)[0]
    R = np.nonzero(rc != 0)[0]
    x = x0.copy()
    x[cc == 1] = lb[cc == 1]
    x[cc == 2] = ub[cc == 2]
    B = np.nonzero(cc != 0)[0]
    A_RF = A[np.ix_(R, F)]
    nF, nR = len(F), len(R)
    K = np.zeros((nF + nR, nF + nR))
    K[np.arange(nF), np.arange(nF)] = p[F]
    K[:nF, nF:] = -A_RF.T
    K[nF:, :nF] = A_RF
    r = np.concatenate([-q[F], np.where(rc[R] == 1, bl[R], bu[R]) - A[np.ix_(R, B)] @ x[B]])
    try:
        s = np.linalg.solve(K, r) if nF + nR else np.zeros(0)
    except np.linalg.LinAlgError:
        s = None
    if s is not None and np.all(np.isfinite(s)):
        x[F] = s[:nF]
        y = np.zeros(len(bl))
        y[R] = s[nF:]
        if _certified(A, bl, bu, lb, ub, q, p, x, y, cc, rc):
            STATS["solves"] += 1
            STATS["rounds"] += 1
            return x, True
    xp, _, rounds = certified_polish(A, bl, bu, lb, ub, q, p, x0, cs, rs)
    STATS["solves"] += 1
    STATS["rounds"] += rounds
    return xp, True
