"""EF bundles (``bundles_per_rank``): each rank's scenarios grouped into bundles
whose subproblem is the extensive form of its members (the reference's
``SPBase._assign_bundles`` spbase.py:219-253, ``SPOpt.subproblem_creation`` /
``FormEF`` spopt.py:743-836, objective normalised by the bundle probability,
sputils.py:273-275).

PH itself stays per scenario, as in the reference: x-bar, W, rho and the
convergence metric are the scenario-level device arrays of the SPBase object
(its context's reductions run on them unchanged).  Only the SOLVE changes:

* the bundles are one more batch on the device (``batch.bundle_batch``: shared
  nonant columns, member blocks, costs weighted by p_s / p_bundle) with its own
  phx context, so the same solvers (lane / workgroup / sparse / generic, chosen
  by its size) serve them;
* before each solve, W and rho are aggregated per bundle -- the weighted sums
  sum_s (p_s / p_bundle) W_s, ... -- which makes the bundle lane's PH terms
  W_b z + rho_b / 2 |z - xbar|^2 + const equal to the EF's sum of its members'
  terms (every member shares the bundle's nonants z); the sums are fixed-order
  (a gather and a reduction over the member axis), so runs are reproducible;
* after it, each scenario's full x is gathered from its member block of the
  bundle solution (nonants: the shared columns), its status and iterations
  from its bundle, and its objective (with its own PH terms) evaluated by the
  scenario context (phx_objective) -- what Ebound / Eobjective / E1 read.
"""
import ctypes

import numpy as np
import torch

from . import _native
from .batch import bundle_batch


def assign_bundles(n_local, bundles_per_rank):
    """Local index slices of this rank's bundles (spbase.py:243-253)."""
    avg = n_local / bundles_per_rank
    return [list(range(int(i * avg), int((i + 1) * avg))) for i in range(bundles_per_rank)]


class BundleSolver:
    def __init__(self, opt, groups):
        b = opt.batch
        self.opt = opt
        self.groups = groups
        self.G = len(groups)
        probs = np.asarray(b.prob, dtype=np.float64)
        bb, members, wts, colmap = bundle_batch(b, groups, probs)
        bb.compress()
        self.batch = bb
        self.K = members.shape[1]
        dev = opt.device
        f64, i32, i64 = torch.float64, torch.int32, torch.int64
        t = lambda a, dt: torch.as_tensor(np.ascontiguousarray(a), dtype=dt).to(dev)   # noqa: E731
        G, K, N, S = self.G, self.K, b.nonant.N, b.S
        # ---- the bundles' problem in their own context
        d = {"rowptr": t(bb.rowptr, i32), "colidx": t(bb.colidx, i32), "kvar": t(bb.kvar, i32),
             "Aconst": t(bb.Aconst, f64), "Avar": t(bb.Avar.ravel() if bb.nvar else np.zeros(1), f64),
             "c": t(bb.minor(bb.c * (1.0 if opt.is_minimizing else -1.0), bb.c_vary), f64),
             "lb": t(bb.minor(bb.lb, bb.bnd_vary), f64), "ub": t(bb.minor(bb.ub, bb.bnd_vary), f64),
             "bl": t(bb.minor(bb.bl, bb.rhs_vary), f64), "bu": t(bb.minor(bb.bu, bb.rhs_vary), f64),
             "slot_col": t(bb.nonant.slot_col, i32)}
        self._dev = d
        lib = opt._native
        ctx = ctypes.c_void_p()
        lib.check(None, lib.create(int(dev.index or 0), ctypes.byref(ctx)), "create (bundles)")
        self.ctx = ctx.value
        import weakref
        weakref.finalize(self, lib.destroy, self.ctx)
        desc = _native.ProblemDesc()
        desc.S, desc.n, desc.m, desc.nnz, desc.N, desc.nvar = G, bb.n, bb.m, bb.nnz, N, bb.nvar
        for k, v in d.items():
            setattr(desc, k, v.data_ptr())
        desc.c_vary, desc.bnd_vary, desc.rhs_vary = int(bb.c_vary), int(bb.bnd_vary), int(bb.rhs_vary)
        lib.check(self.ctx, lib.set_problem(self.ctx, desc), "set_problem (bundles)")
        self._desc = desc
        # ---- outputs and PH-term arrays of the bundle lanes
        self.x = torch.zeros(bb.n * G, dtype=f64, device=dev)
        self.y = torch.zeros(max(bb.m, 1) * G, dtype=f64, device=dev)
        self.obj = torch.zeros(G, dtype=f64, device=dev)
        self.status = torch.zeros(G, dtype=i32, device=dev)
        self.iters = torch.zeros(G, dtype=i32, device=dev)
        self.W = torch.zeros(max(N, 1) * G, dtype=f64, device=dev)
        self.rho = torch.zeros(max(N, 1) * G, dtype=f64, device=dev)
        # ---- index maps (all fixed-order gathers)
        self._members = t(members.ravel(), i64)                   # (G K)
        self._wts = t(wts, f64)                                   # (G, K)
        xi = opt._xbar_idx.reshape(N, S) if N else np.zeros((0, S), dtype=np.int32)
        self.xbar_idx = t(xi[:, members[:, 0]].ravel(), i32)     # (N, G): the members' node slots
        bundle_of = np.zeros(S, dtype=np.int64)
        slot_of = np.zeros(S, dtype=np.int64)
        for g, grp in enumerate(groups):
            for r, s in enumerate(grp):
                bundle_of[s], slot_of[s] = g, r
        self._bundle_of = t(bundle_of, i64)
        # x of scenario s, column j  <-  bundle column colmap[slot_of[s], j] of bundle_of[s]
        gx = colmap[slot_of, :].T * G + bundle_of[None, :]       # (n, S)
        self._gx = t(gx.ravel(), i64)

    def _aggregate(self, src, dst):
        """dst[t, g] = sum_r w[g, r] src[t, members[g, r]] (fixed order)."""
        N, S = self.opt.batch.nonant.N, self.opt.batch.S
        if N == 0:
            return
        v = src.view(N, S).index_select(1, self._members).view(N, self.G, self.K)
        dst.view(N, self.G).copy_((v * self._wts).sum(dim=2))

    def solve(self, so):
        """One batched solve of every local bundle; the scenario-level x, status,
        iterations and objectives of the SPBase object from it."""
        opt = self.opt
        lib = opt._native
        N = opt.batch.nonant.N
        W_on, prox_on = bool(opt.W_on and N), bool(opt.prox_on and N)
        if W_on:
            self._aggregate(opt._W, self.W)
        if prox_on:
            self._aggregate(opt._rho, self.rho)
        st = opt._stream()
        lib.check(self.ctx, lib.set_ph_terms(self.ctx, self.W.data_ptr() if W_on else None,
                                             self.rho.data_ptr() if prox_on else None,
                                             opt._xbar_node.data_ptr() if prox_on else None,
                                             self.xbar_idx.data_ptr() if prox_on else None,
                                             int(W_on), int(prox_on), st), "set_ph_terms (bundles)")
        so.defer = 0
        total = ctypes.c_int32(0)
        lib.check(self.ctx, lib.solve(self.ctx, ctypes.byref(so), self.x.data_ptr(), self.y.data_ptr(),
                                      self.obj.data_ptr(), self.status.data_ptr(), self.iters.data_ptr(),
                                      ctypes.byref(total), st), "solve (bundles)")
        opt._x.copy_(self.x.index_select(0, self._gx))
        opt._status.copy_(self.status.index_select(0, self._bundle_of))
        opt._iters.copy_(self.iters.index_select(0, self._bundle_of))
        # each scenario's own objective, PH terms included (the scenario context's)
        opt._set_ph_terms()
        lib.check(opt._ctx, lib.objective(opt._ctx, opt._x.data_ptr(), opt._obj.data_ptr(), st), "objective")
        return int(total.value)
