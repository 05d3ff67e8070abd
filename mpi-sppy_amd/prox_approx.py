"""Linearised proximal terms (options ``linearize_proximal_terms``,
``proximal_linearization_tolerance`` (default 0.1), ``initial_proximal_cut_count``
(default 2)): the reference's outer approximation of the prox term's x^2 by
tangent cuts (``PHBase.attach_PH_to_objective`` phbase.py:617-699,
``_update_prox_approx`` :570-582, ``ProxApproxManagerContinuous``
utils/prox_approx.py:1-180).

Per nonant slot t a subproblem gains a column xsq_t >= 0 and one row per cut
point a, xsq_t - 2 a x_t >= -a^2 (the tangent of x^2 at a); its prox term is
rho/2 (xsq_t - 2 xbar x_t + xbar^2), so every prox-on subproblem is an LP.  The
cut points start at lb (if lb != 0) and ub (if ub != 0 and lb != ub), plus
initial_proximal_cut_count - 2 evenly spaced interior points; before every
prox-on solve, each (scenario, slot) whose last solution has x^2 - xsq > tol
gets a cut at the Newton projection of (x, xsq) onto y = x^2 (the reference's
iteration, math.isclose at 1e-6 rel / abs).

Device side: the same LP in its incremental form, in a phx context of its
own (as the EF bundles).  With the tangent at 0 standing for xsq >= 0, the
envelope phi(x) = max(0, max_k tangent_k(x)) is piecewise linear on [lb, ub]
with increasing slopes 2 a_i between the breakpoints (a_i + a_{i+1}) / 2, so
the prox-on subproblem is: columns [x (n) | delta (N x Kp)], rows [A (m) |
x_t - sum_i delta_ti = lb_t (N)], delta_ti in [0, segment length], cost of
delta_ti rho/2 * 2 a_i (as linear PH terms of that context: slot t, the nonant
column, gets W_on W - rho xbar; the delta slots get rho a_i), constant rho/2
phi(lb).  An optimum fills the segments in order (increasing slopes), so x is
the optimum of the reference's LP and xsq = phi(x) its xsq.  This form has one
row per nonant and no near-parallel cut rows however many cuts accumulate (the
cut-row form made the KKT systems degenerate and the lane limits overflow).
Kp, the segment slots per nonant, is the next power of two holding the most
cut points any scenario has (at least 4, zero-length segments pad); the
context is rebuilt when a cut is added (the JIT kernel is cached by its
source text, which changes only with Kp).

Prox-off solves (Iter0, the W-only bounds) never see the cuts: xsq has zero
cost there, so x is the plain LP's; they run on the scenario context and xsq
takes its least feasible value phi(x) -- the value a simplex basis gives it
(basic on the binding tangent, else nonbasic at 0).

Binary nonants (``linearize_binary_proximal_terms``) do not arise: the engine's
subproblems are LPs / QPs over continuous variables.
"""
import ctypes
import weakref

import numpy as np
import torch

from . import _native
from .batch import BatchData, NonantSpec


def initial_points(lb, ub, count):
    """``ProxApproxManagerContinuous._create_initial_cuts`` (prox_approx.py:124-141)."""
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


def _isclose(a, b):
    return np.abs(a - b) <= np.maximum(1e-6 * np.maximum(np.abs(a), np.abs(b)), 1e-6)


def newton_project(xp, yp):
    """``check_tol_add_cut``'s Newton iteration (prox_approx.py:84-116), element
    by element: the point of y = x^2 nearest (xp, yp), stepped from xp until two
    iterates are math.isclose(rel_tol=1e-6, abs_tol=1e-6); the last iterate."""
    xp = np.asarray(xp, dtype=np.float64)
    yp = np.asarray(yp, dtype=np.float64)

    def step(v):
        return v - (v * (1 - 2 * yp + 2 * v * v) - xp) / (1 + 6 * v * v - 2 * yp)

    this = xp.copy()
    nxt = step(this)
    done = _isclose(this, nxt)
    for _ in range(1000):
        if done.all():
            break
        this = np.where(done, this, nxt)
        nxt = np.where(done, nxt, step(this))
        done = _isclose(this, nxt)
    return nxt


def _pad_point(lb, ub):
    return ub + np.maximum(1.0, ub - lb)


class ProxLinSolver:
    def __init__(self, opt, tol, initial_count):
        b = opt.batch
        nn = b.nonant
        self.opt = opt
        self.tol = float(tol)
        S, n, N = b.S, b.n, nn.N
        self.S, self.n, self.N = S, n, N
        lb = np.broadcast_to(np.asarray(b.lb, dtype=np.float64), (S, n))
        ub = np.broadcast_to(np.asarray(b.ub, dtype=np.float64), (S, n))
        cols = np.asarray(nn.slot_col, dtype=np.int64)
        self.lbn = np.ascontiguousarray(lb[:, cols])          # (S, N)
        self.ubn = np.ascontiguousarray(ub[:, cols])
        if not (np.isfinite(self.lbn).all() and np.isfinite(self.ubn).all()):
            raise RuntimeError("linearize_nonbinary_proximal_terms requires all "
                               "nonanticipative variables to have bounds")
        # cut points (S, N, cap) and counts (S, N)
        init = [[initial_points(self.lbn[s, t], self.ubn[s, t], int(initial_count)) for t in range(N)]
                for s in range(S)]
        cap = max(4, max((len(p) for row in init for p in row), default=0))
        self.pts = np.zeros((S, N, cap))
        self.cnt = np.zeros((S, N), dtype=np.int64)
        for s in range(S):
            for t in range(N):
                p = init[s][t]
                self.pts[s, t, :len(p)] = p
                self.cnt[s, t] = len(p)
        self.xsq = torch.zeros(max(N, 1) * S, dtype=torch.float64, device=opt.device)
        self.xsq_stale = True           # xsq of the last solve not yet known (prox-off solve)
        self.have_solution = False
        self.ctx = None
        self.cuts_added = 0
        self.cuts_built = -1
        self.rebuilds = 0

    # ---- cut bookkeeping (host)
    def _x_nonants(self):
        opt = self.opt
        S, N = self.S, self.N
        cols = torch.as_tensor(np.asarray(opt.batch.nonant.slot_col, dtype=np.int64), device=opt.device)
        return opt._x.view(-1, S).index_select(0, cols)          # (N, S)

    def envelope(self, xn):
        """max(0, max_k tangent_k(x)) per (slot, scenario): xn (N, S) numpy."""
        a = self.pts.transpose(1, 0, 2)                            # (N, S, cap)
        valid = np.arange(a.shape[2])[None, None, :] < self.cnt.T[:, :, None]
        tang = np.where(valid, 2.0 * a * xn[:, :, None] - a * a, -np.inf)
        return np.maximum(0.0, tang.max(axis=2))

    def refresh_xsq(self):
        """xsq of the last solve: phi(x), its least feasible value (the LP's
        own value of it after a prox-on solve)."""
        if not self.xsq_stale:
            return
        xn = self._x_nonants().cpu().numpy()
        self.xsq.copy_(torch.as_tensor(self.envelope(xn).ravel(), device=self.xsq.device))
        self.xsq_stale = False

    def add_cuts(self):
        """``_update_prox_approx`` (phbase.py:570-582): a cut at the Newton
        projection of the last (x, xsq) wherever x^2 - xsq > tol."""
        self.refresh_xsq()
        xn = self._x_nonants().cpu().numpy().T                     # (S, N)
        ys = self.xsq.view(self.N, self.S).cpu().numpy().T
        viol = (xn * xn - ys) > self.tol
        if not viol.any():
            return 0
        ss, tt = np.nonzero(viol)
        a = newton_project(xn[ss, tt], ys[ss, tt])
        need = int(self.cnt.max()) + 1
        if need > self.pts.shape[2]:
            grow = np.zeros((self.S, self.N, max(need, 2 * self.pts.shape[2])))
            grow[:, :, :self.pts.shape[2]] = self.pts
            self.pts = grow
        self.pts[ss, tt, self.cnt[ss, tt]] = a
        self.cnt[ss, tt] += 1
        self.cuts_added += len(ss)
        return len(ss)

    # ---- the LP in its own context
    def _segments(self):
        """The envelope phi(x) = max(0, max_k tangent_k(x)) on [lb, ub] as
        segments: points P (S, N, Kp) sorted with 0 (the xsq >= 0 bound, the
        tangent at 0) and +inf padding; tangent i is the active one between
        the breakpoints (P_{i-1} + P_i)/2 and (P_i + P_{i+1})/2; its segment,
        clipped to [lb, ub], has slope 2 P_i.  Returns (lengths, slopes,
        phi(lb)), each (S, N, Kp) / (S, N)."""
        cap = self.pts.shape[2]
        valid = np.arange(cap)[None, None, :] < self.cnt[:, :, None]
        P = np.concatenate([np.zeros(self.cnt.shape + (1,)), np.where(valid, self.pts, np.inf)], axis=2)
        P = np.sort(P, axis=2)
        Kp = 4
        while Kp < P.shape[2]:
            Kp *= 2
        P = np.pad(P, ((0, 0), (0, 0), (0, Kp - P.shape[2])), constant_values=np.inf)
        with np.errstate(invalid="ignore"):
            brk = 0.5 * (P[:, :, :-1] + P[:, :, 1:])                    # (S, N, Kp-1), inf past the points
        lo, hi = self.lbn[:, :, None], self.ubn[:, :, None]
        edges = np.concatenate([lo, np.clip(np.nan_to_num(brk, nan=np.inf), lo, hi), hi], axis=2)
        lengths = np.diff(edges, axis=2)                               # (S, N, Kp)
        slopes = np.where(np.isfinite(P), 2.0 * P, 0.0)
        with np.errstate(invalid="ignore"):
            tl = np.where(np.isfinite(P), 2.0 * P * self.lbn[:, :, None] - P * P, -np.inf)
        return lengths, slopes, tl.max(axis=2)

    def _build(self, lengths):
        """(Re)create the context: columns [x (n) | delta (N x Kp)], rows
        [A (m) | x_t - sum_i delta_ti = lb_t (N)], delta_ti in [0, length_ti]."""
        opt = self.opt
        b = opt.batch
        S, n, m, N = self.S, self.n, b.m, self.N
        Kp = lengths.shape[2]
        cols = np.asarray(b.nonant.slot_col, dtype=np.int64)
        rowptr = list(b.rowptr)
        colidx = list(b.colidx)
        nnz0 = b.nnz
        for t in range(N):
            colidx += [int(cols[t])] + [n + t * Kp + i for i in range(Kp)]
            rowptr.append(len(colidx))
        Alink = np.tile(np.concatenate([[1.0], -np.ones(Kp)]), (S, N))
        A = np.concatenate([np.asarray(b.A_full, dtype=np.float64).reshape(S, nnz0), Alink], axis=1)

        def per(v, w):
            v = np.asarray(v, dtype=np.float64)
            return v if v.ndim == 2 else np.broadcast_to(v, (S, w))

        bl = np.concatenate([per(b.bl, m), self.lbn], axis=1)
        bu = np.concatenate([per(b.bu, m), self.lbn], axis=1)
        lb = np.concatenate([per(b.lb, n), np.zeros((S, N * Kp))], axis=1)
        ub = np.concatenate([per(b.ub, n), lengths.reshape(S, N * Kp)], axis=1)
        c = np.concatenate([per(b.c, n), np.zeros((S, N * Kp))], axis=1)
        slot_col = np.concatenate([cols, n + np.arange(N * Kp)])
        spec = NonantSpec(slot_col, np.ones(len(slot_col), dtype=np.int32), np.arange(len(slot_col)), [None],
                          [np.ones(S)], ["v%d" % t for t in range(len(slot_col))])
        bb = BatchData(["s%d" % s for s in range(S)], rowptr, colidx, A, bl, bu, lb, ub, c,
                       np.zeros(S), b.sense, np.full(S, 1.0 / S), spec)
        bb.compress(force_rhs_vary=True)
        if not bb.bnd_vary:                                            # (the structure must not depend on
            bb.lb = np.broadcast_to(bb.lb, (S, bb.n)).copy()           #  the segment lengths)
            bb.ub = np.broadcast_to(bb.ub, (S, bb.n)).copy()
            bb.bnd_vary = True
        dev = opt.device
        f64, i32 = torch.float64, torch.int32
        t_ = lambda v, dt: torch.as_tensor(np.ascontiguousarray(v), dtype=dt).to(dev)   # noqa: E731
        sgn = 1.0 if opt.is_minimizing else -1.0
        d = {"rowptr": t_(bb.rowptr, i32), "colidx": t_(bb.colidx, i32), "kvar": t_(bb.kvar, i32),
             "Aconst": t_(bb.Aconst, f64), "Avar": t_(bb.Avar.ravel() if bb.nvar else np.zeros(1), f64),
             "c": t_(bb.minor(bb.c * sgn, bb.c_vary), f64),
             "lb": t_(bb.minor(bb.lb, bb.bnd_vary), f64), "ub": t_(bb.minor(bb.ub, bb.bnd_vary), f64),
             "bl": t_(bb.minor(bb.bl, bb.rhs_vary), f64), "bu": t_(bb.minor(bb.bu, bb.rhs_vary), f64),
             "slot_col": t_(bb.nonant.slot_col, i32)}
        lib = opt._native
        ctx = ctypes.c_void_p()
        lib.check(None, lib.create(int(dev.index or 0), ctypes.byref(ctx)), "create (linearised prox)")
        desc = _native.ProblemDesc()
        desc.S, desc.n, desc.m, desc.nnz, desc.N, desc.nvar = S, bb.n, bb.m, bb.nnz, len(slot_col), bb.nvar
        for k, v in d.items():
            setattr(desc, k, v.data_ptr())
        desc.c_vary, desc.bnd_vary, desc.rhs_vary = int(bb.c_vary), int(bb.bnd_vary), int(bb.rhs_vary)
        lib.check(ctx.value, lib.set_problem(ctx.value, desc), "set_problem (linearised prox)")
        if self.ctx is not None:
            self._finalizer()
        self.ctx = ctx.value
        self._finalizer = weakref.finalize(self, lib.destroy, self.ctx)
        self._dev = d
        self.rebuilds += 1
        self.Kp = Kp
        self.xl = torch.zeros(bb.n * S, dtype=f64, device=dev)
        self.yl = torch.zeros(max(bb.m, 1) * S, dtype=f64, device=dev)
        self.obj = torch.zeros(S, dtype=f64, device=dev)
        self.W2 = torch.zeros(len(slot_col) * S, dtype=f64, device=dev)

    # ---- one prox-on solve
    def solve(self, so):
        """The reference's LP, min c'x + W x + rho/2 (xsq - 2 xbar x) s.t. xsq >=
        every tangent, xsq >= 0, in its incremental form: xsq = phi(x) =
        phi(lb) + sum_i slope_i delta_i with x_t = lb_t + sum_i delta_i (the
        slopes increase, so an optimum fills the segments in order and
        reproduces phi).  No near-parallel cut rows, one row per nonant."""
        opt = self.opt
        S, N, n = self.S, self.N, self.n
        if self.have_solution:
            self.add_cuts()
        if self.ctx is None or self.cuts_built != self.cuts_added:
            lengths, slopes, _ = self._segments()
            self._build(lengths)
            self._slopes = torch.as_tensor(np.ascontiguousarray(slopes.transpose(1, 2, 0)),
                                           device=opt.device)              # (N, Kp, S)
            self.cuts_built = self.cuts_added
        Kp = self.Kp
        lib = opt._native
        st = opt._stream()
        W2 = self.W2.view(-1, S)
        xb = opt._xbar_node.index_select(0, opt._xbar_idx_t.long()).view(N, S)
        rho = opt._rho.view(N, S)
        W2[:N].copy_(-rho * xb)
        if opt.W_on:
            W2[:N].add_(opt._W.view(N, S))
        W2[N:].view(N, Kp, S).copy_(0.5 * rho[:, None, :] * self._slopes)
        lib.check(self.ctx, lib.set_ph_terms(self.ctx, self.W2.data_ptr(), None, None, None, 1, 0, st),
                  "set_ph_terms (linearised prox)")
        so.defer = 0
        total = ctypes.c_int32(0)
        lib.check(self.ctx, lib.solve(self.ctx, ctypes.byref(so), self.xl.data_ptr(), self.yl.data_ptr(),
                                      self.obj.data_ptr(), opt._status.data_ptr(), opt._iters.data_ptr(),
                                      ctypes.byref(total), st), "solve (linearised prox)")
        opt._x.copy_(self.xl[:n * S])
        self.xsq_stale = True            # xsq = phi(x), the LP's value of it
        self.have_solution = True
        self.objective_into(opt._obj)
        return int(total.value)

    def after_plain_solve(self):
        """A prox-off solve on the scenario context replaced x."""
        self.xsq_stale = True
        self.have_solution = True

    def objective_into(self, out):
        """Each scenario's objective with the linearised PH terms (min sense, c0
        excluded): c'x + W_on W x + prox_on rho/2 (xsq - 2 xbar x + xbar^2)."""
        opt = self.opt
        S, N = self.S, self.N
        lib = opt._native
        st = opt._stream()
        lib.check(opt._ctx, lib.set_ph_terms(opt._ctx, None, None, None, None, 0, 0, st), "set_ph_terms")
        lib.check(opt._ctx, lib.objective(opt._ctx, opt._x.data_ptr(), out.data_ptr(), st), "objective")
        opt._set_ph_terms()
        xn = self._x_nonants()
        if opt.W_on:
            out.add_((opt._W.view(N, S) * xn).sum(dim=0))
        if opt.prox_on:
            self.refresh_xsq()
            xb = opt._xbar_node.index_select(0, opt._xbar_idx_t.long()).view(N, S)
            rho = opt._rho.view(N, S)
            out.add_((0.5 * rho * (self.xsq.view(N, S) - 2.0 * xb * xn + xb * xb)).sum(dim=0))
