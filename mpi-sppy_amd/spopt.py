"""SPOpt — batched subproblem solves and expectation reductions.

Mirrors ``mpisppy.spopt.SPOpt`` (``mpisppy/spopt.py``): ``solve_loop``
(226-307) with the same hook calls (``pre_solve_loop`` / per-subproblem
``pre_solve`` / ``post_solve`` / ``post_solve_loop``), ``Eobjective`` (310-343),
``Ebound`` (346-391), ``_update_E1`` (394-408), ``feas_prob`` / ``infeas_prob``
(411-466).  Where the reference loops over scenarios calling an external solver
(``solve_one`` 85-223), this calls ONE native batched solve for all local
scenarios (``phx_solve``: PDHG + KKT polish on the GPU).

Solver knobs come from the ``solver_options`` dict exactly where the reference
passes solver options (``iter0_solver_options`` / ``iterk_solver_options``,
phbase.py:273-275): keys ``pdhg_max_iters``, ``pdhg_check_every``,
``pdhg_restart_max``, ``polish``, ``polish_refine``, ``polish_below``,
``kkt_tol``, ``opt_tol``, ``polish_reg``, ``warm_start``, ``ipm_after``,
``ipm_max_it``, ``ipm_tol``, ``lane_solver``, ``as_rounds``, ``warm_passes``.
"""
import ctypes
import inspect
import time

import numpy as np
import torch

from . import _native
from .spbase import SPBase

SOLVER_DEFAULTS = {
    "pdhg_max_iters": 200000,
    "pdhg_check_every": 64,
    "pdhg_restart_max": 1000,
    "polish": 1,
    "polish_refine": 10,
    "polish_below": 1e-4,
    "opt_tol": 1e-8,
    "kkt_tol": 1e-9,
    "polish_reg": 1e-6,
    "warm_start": 1,
    "ipm_after": 1024,
    "ipm_max_it": 60,
    "ipm_tol": 1e-10,
    "lane_solver": 1,
    "as_rounds": 4,
    "warm_passes": 1,
}

OPTIMAL, ITER_LIMIT, NUMERIC_FAIL = 1, 2, 3


def _overrides(obj, name):
    """True if obj's class overrides hook ``name`` of its extension base."""
    from .extensions.extension import Extension
    f = getattr(type(obj), name, None)
    return f is not None and f is not getattr(Extension, name, None)


class SPOpt(SPBase):
    def __init__(self, options, all_scenario_names, scenario_creator, scenario_denouement=None,
                 all_nodenames=None, mpicomm=None, extensions=None, extension_kwargs=None,
                 scenario_creator_kwargs=None, variable_probability=None, E1_tolerance=1e-5,
                 _native_lib=None, _device=None):
        super().__init__(options, all_scenario_names, scenario_creator,
                         scenario_denouement=scenario_denouement, all_nodenames=all_nodenames,
                         mpicomm=mpicomm, scenario_creator_kwargs=scenario_creator_kwargs,
                         variable_probability=variable_probability, E1_tolerance=E1_tolerance,
                         _native_lib=_native_lib, _device=_device)
        self.current_solver_options = None
        self.extensions = extensions
        self.extension_kwargs = extension_kwargs
        self.W_on = 0
        self.prox_on = 0
        self.solve_stats = []
        self._solve_pending = False
        if self.extensions is not None:
            if self.extension_kwargs is None:
                self.extobject = self.extensions(self)
            else:
                self.extobject = self.extensions(self, **self.extension_kwargs)

    # ------------------------------------------------------------ solve
    def _solve_opts(self, solver_options):
        o = dict(SOLVER_DEFAULTS)
        if solver_options:
            for k, v in solver_options.items():
                if k in o:
                    o[k] = v
        so = _native.SolveOpts()
        so.max_iters = int(o["pdhg_max_iters"])
        so.check_every = int(o["pdhg_check_every"])
        so.restart_max = int(o["pdhg_restart_max"])
        so.polish = int(o["polish"])
        so.refine_steps = int(o["polish_refine"])
        so.warm_start = int(o["warm_start"])
        so.polish_below = float(o["polish_below"])
        so.opt_tol = float(o["opt_tol"])
        so.kkt_tol = float(o["kkt_tol"])
        so.reg = float(o["polish_reg"])
        so.ipm_after = int(o["ipm_after"])
        so.ipm_max_it = int(o["ipm_max_it"])
        so.ipm_tol = float(o["ipm_tol"])
        so.lane_solver = int(o["lane_solver"])
        so.as_rounds = int(o["as_rounds"])
        so.warm_passes = int(o["warm_passes"])
        return so

    def _set_ph_terms(self):
        """Push the active PH objective terms (W_on/prox_on) to the native context."""
        lib = self._native
        N = self.batch.nonant.N
        W = self._W.data_ptr() if (self.W_on and N) else None
        rho = self._rho.data_ptr() if (self.prox_on and N) else None
        xb = self._xbar_node.data_ptr() if (self.prox_on and N) else None
        xi = self._xbar_idx_t.data_ptr() if (self.prox_on and N) else None
        lib.check(self._ctx, lib.set_ph_terms(self._ctx, W, rho, xb, xi, int(self.W_on and N > 0),
                                              int(self.prox_on and N > 0), self._stream()), "set_ph_terms")

    def solve_loop(self, solver_options=None, use_scenarios_not_subproblems=False, dtiming=False,
                   gripe=False, disable_pyomo_signal_handling=False, tee=False, verbose=False):
        """Batched solve of every local subproblem (spopt.py:226-307)."""
        if self.extensions is not None:
            self.extobject.pre_solve_loop()
            if _overrides(self.extobject, "pre_solve"):
                for s in self.local_subproblems.values():
                    self.extobject.pre_solve(s)
        self._settle()
        lib = self._native
        so = self._solve_opts(solver_options)
        # Without extensions nothing reads per-scenario results right after the
        # solve, so it is deferred: phx_solve returns once the lane kernels are
        # enqueued and the next PH step's reductions queue behind them; every
        # reader of solve results calls _settle() (convergence_diff finishes it
        # and redoes the step in the rare case a scenario needed the generic path).
        defer = (self.extensions is None and not dtiming and so.lane_solver
                 and bool((solver_options or {}).get("defer", 1)))
        so.defer = 1 if defer else 0
        self._set_ph_terms()
        total = ctypes.c_int32(0)
        t0 = time.perf_counter()
        lib.check(self._ctx, lib.solve(self._ctx, ctypes.byref(so), self._x.data_ptr(), self._y.data_ptr(),
                                       self._obj.data_ptr(), self._status.data_ptr(), self._iters.data_ptr(),
                                       ctypes.byref(total), self._stream()), "solve")
        self._conv_cache = None
        self._bump()
        rec = {"wall_s": None, "t0": t0, "gripe": gripe}
        self.solve_stats.append(rec)
        if total.value == -1:
            self._solve_pending = True
        else:
            self._record_solve(rec, int(total.value), 0)
        if self.extensions is not None:
            if _overrides(self.extobject, "post_solve"):
                for s in self.local_subproblems.values():
                    self.extobject.post_solve(s, None)
            self.extobject.post_solve_loop()
        if dtiming:
            allt = self.mpicomm.gather(self.solve_stats[-1]["wall_s"])
            if self.cylinder_rank == 0:
                print("Batched solve times (seconds): min=%4.2f mean=%4.2f max=%4.2f"
                      % (min(allt), sum(allt) / len(allt), max(allt)))

    def _record_solve(self, rec, total, stragglers):
        lib = self._native
        stt = _native.SolveStats()
        lib.check(self._ctx, lib.last_solve_stats(self._ctx, ctypes.byref(stt)), "last_solve_stats")
        n_bad = int(stt.not_optimal)
        t0, gripe = rec.pop("t0"), rec.pop("gripe")
        rec.update({"pdhg_iters": total, "pdhg_ms": stt.pdhg_ms, "launches": stt.pdhg_launches,
                    "lane_iters": stt.lane_iters, "polish_ms": stt.polish_ms, "ipm_ms": stt.ipm_ms,
                    "lane_ms": stt.lane_ms, "lane_warm_ms": stt.lane_warm_ms,
                    "lane_warm_list_ms": stt.lane_warm_list_ms, "lane_certified": stt.lane_certified,
                    "lane_warm_certified": stt.lane_warm_certified, "stragglers": stragglers,
                    "wall_s": time.perf_counter() - t0, "not_optimal": n_bad})
        if n_bad and gripe:
            stc = self._status.cpu().numpy()
            name = self.__class__.__name__
            if self.spcomm:
                name = self.spcomm.__class__.__name__
            for k in np.nonzero(stc != OPTIMAL)[0][:10]:
                print("[%s] Solve failed for scenario %s" % (name, self.local_scenario_names[k]))
                print("status=", {ITER_LIMIT: "iteration limit", NUMERIC_FAIL: "numerical failure"}.get(
                    int(stc[k]), int(stc[k])))

    def _sync_solve(self):
        """Finish a deferred solve (phx_solve_finish); returns the number of local
        scenarios that needed the generic path (their x changed)."""
        if not self._solve_pending:
            return 0
        lib = self._native
        strag = ctypes.c_int32(0)
        total = ctypes.c_int32(0)
        lib.check(self._ctx, lib.solve_finish(self._ctx, ctypes.byref(strag), ctypes.byref(total)),
                  "solve_finish")
        self._solve_pending = False
        self._record_solve(self.solve_stats[-1], int(total.value), int(strag.value))
        if strag.value:
            self._bump()
        return int(strag.value)

    def _settle(self):
        """Make solve results and W final before anything reads them."""
        if self._solve_pending or getattr(self, "_w_uncommitted", False):
            self._settle_pending()

    def _settle_pending(self):
        self._sync_solve()

    # ------------------------------------------------------------ expectations
    def _expect(self, values):
        self._settle()
        lib = self._native
        lib.check(self._ctx, lib.expect(self._ctx, self._prob.data_ptr(), values.data_ptr(),
                                        self._status.data_ptr(), self._expect_buf.data_ptr(),
                                        self._stream()), "expect")
        return self._expect_buf

    def Eobjective(self, verbose=False):
        """sum_s p_s * objective_s incl. active W/prox terms (spopt.py:310-343)."""
        self._objective_now()
        buf = self._expect(self._obj_eval).clone()
        g = self.mpicomm.allreduce_(buf[0:1].clone())
        v = float(g.item())
        return v if self.is_minimizing else -v

    def _objective_now(self):
        """Objective of the current x under the current W/xbar/rho and W_on/prox_on."""
        self._settle()
        if not hasattr(self, "_obj_eval"):
            self._obj_eval = torch.zeros_like(self._obj)
        self._set_ph_terms()
        lib = self._native
        lib.check(self._ctx, lib.objective(self._ctx, self._x.data_ptr(), self._obj_eval.data_ptr(),
                                           self._stream()), "objective")

    def Ebound(self, verbose=False, extra_sum_terms=None):
        """sum_s p_s * outer_bound_s (+ extra terms), spopt.py:346-391."""
        buf = self._expect(self._outer)
        loc = [float(buf[0].item())]
        if extra_sum_terms is not None:
            loc += list(extra_sum_terms)
        t = torch.tensor(loc, dtype=torch.float64, device=self.device)
        self.mpicomm.allreduce_(t)
        sgn = 1.0 if self.is_minimizing else -1.0
        if extra_sum_terms is None:
            return sgn * float(t[0].item())
        return sgn * float(t[0].item()), t[1:].cpu().numpy()

    def _update_E1(self):
        buf = self._expect(self._outer)
        t = buf[1:2].clone()
        self.mpicomm.allreduce_(t)
        self.E1 = float(t.item())

    def feas_prob(self):
        buf = self._expect(self._outer)
        t = buf[2:3].clone()
        self.mpicomm.allreduce_(t)
        return float(t.item())

    def infeas_prob(self):
        buf = self._expect(self._outer)
        t = (buf[1:2] - buf[2:3]).clone()
        self.mpicomm.allreduce_(t)
        return float(t.item())

    def subproblem_creation(self, verbose=False):
        """No bundles: subproblems are the scenarios (spopt.py:805-836)."""
        self.local_subproblems = self.local_scenarios

    def _create_solvers(self, presolve=True):
        """The native context built in SPBase already holds the batched 'solver'."""
        return None
