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
``ipm_max_it``, ``ipm_tol``, ``lane_solver``, ``as_rounds``, ``warm_passes``, ``wg_warm``, ``wg_first``,
``sp``, ``sp_rounds``, ``seed_templates``, ``rescue_rounds``, ``lane_ipm_tol``.
Two more are read once, when the problem is set up (``SPBase._upload_batch``),
because they are compiled into the structure-specialised lane kernels:
``lane_multi_theta`` (> 0: bounded multi-change active-set updates -- every
violation within theta of the worst -- for ``lane_multi_rounds`` rounds, default
4, after the full updates; 0: single changes, the default) and
``lane_multi_rounds``.
"""
import ctypes
import inspect
import time

import numpy as np
import torch

from . import _native
from .spbase import SPBase
from .views import ScenarioView, ScenarioViews

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
    "wg_warm": 16,
    "sp": 1,
    "sp_rounds": 16,
    "seed_templates": 64,
    "rescue_rounds": 0,
    "lane_ipm_tol": 0.0,
    "wg_first": 0,
}

OPTIMAL, ITER_LIMIT, NUMERIC_FAIL, INFEASIBLE = 1, 2, 3, 4


class SolveResults:
    """What ``post_solve(s, results)`` hooks read from a solver results object
    (spopt.py:166-206 hands Pyomo's to the extensions): ``solver.status``,
    ``solver.termination_condition`` and ``problem.lower_bound/upper_bound``
    (the subproblem's objective at the certified optimum, model sense)."""

    class _NS:
        pass

    _TC = {OPTIMAL: "optimal", ITER_LIMIT: "maxIterations", NUMERIC_FAIL: "error", INFEASIBLE: "infeasible"}

    def __init__(self, status, objective):
        self.solver = SolveResults._NS()
        self.problem = SolveResults._NS()
        tc = SolveResults._TC.get(int(status), "unknown")
        self.solver.termination_condition = tc
        self.solver.status = "ok" if status == OPTIMAL else ("warning" if status == INFEASIBLE else "error")
        ok = status == OPTIMAL
        self.problem.lower_bound = float(objective) if ok else float("nan")
        self.problem.upper_bound = float(objective) if ok else float("nan")

    def __repr__(self):
        return "SolveResults(%s, %r)" % (self.solver.termination_condition, self.problem.upper_bound)


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
        self._make_views()
        if self.extensions is not None:
            if self.extension_kwargs is None:
                self.extobject = self.extensions(self)
            else:
                self.extobject = self.extensions(self, **self.extension_kwargs)

    def _make_views(self):
        self.local_scenarios = ScenarioViews(self, self.local_scenario_names)
        self.local_subproblems = self.local_scenarios

    # ------------------------------------------------------------ solve
    def _solve_opts(self, solver_options):
        """phx_solve_opts from a solver-options dict (cached per dict contents; a
        fresh struct is returned, so callers may modify it)."""
        key = tuple(sorted((k, v) for k, v in (solver_options or {}).items()
                           if k in SOLVER_DEFAULTS and isinstance(v, (int, float))))
        cache = self.__dict__.setdefault("_solve_opts_cache", {})
        so = cache.get(key)
        if so is None:
            so = cache[key] = self._make_solve_opts(solver_options)
        out = _native.SolveOpts()
        ctypes.pointer(out)[0] = so
        return out

    def _make_solve_opts(self, solver_options):
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
        so.wg_warm = int(o["wg_warm"])
        so.sp = int(o["sp"])
        so.sp_rounds = int(o["sp_rounds"])
        so.seed_templates = int(o["seed_templates"])
        so.rescue_rounds = int(o["rescue_rounds"])
        so.lane_ipm_tol = float(o["lane_ipm_tol"])
        so.wg_first = int(o["wg_first"])
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
        self._apply_fixing()
        lib = self._native
        so = self._solve_opts(solver_options)
        # Without extensions nothing reads per-scenario results right after the
        # solve, so it is deferred: phx_solve returns once the lane kernels are
        # enqueued and the next PH step's reductions queue behind them; every
        # reader of solve results calls _settle() (convergence_diff finishes it
        # and redoes the step in the rare case a scenario needed the generic path).
        defer = (self.extensions is None and not dtiming and so.lane_solver and self._bundles is None
                 and self._prox_lin is None and bool((solver_options or {}).get("defer", 1)))
        so.defer = 1 if defer else 0
        self._set_ph_terms()
        total = ctypes.c_int32(0)
        t0 = time.perf_counter()
        self._x_touched = True
        self._solve_ctx = self._ctx
        if self._bundles is not None:
            # EF bundles: one batched solve of the bundles, scenario results from it
            total.value = self._bundles.solve(so)
            self._solve_ctx = self._bundles.ctx
        elif self._prox_lin is not None and self.prox_on and self.batch.nonant.N:
            # linearised prox: the LP with the tangent cuts, in its own context
            total.value = self._prox_lin.solve(so)
            self._solve_ctx = self._prox_lin.ctx
        else:
            lib.check(self._ctx, lib.solve(self._ctx, ctypes.byref(so), self._x.data_ptr(), self._y.data_ptr(),
                                           self._obj.data_ptr(), self._status.data_ptr(), self._iters.data_ptr(),
                                           ctypes.byref(total), self._stream()), "solve")
            if self._prox_lin is not None:
                self._prox_lin.after_plain_solve()
        self._conv_cache = None
        self._bump()
        if getattr(self, "_fix_lb", None) is not None:
            # fixed columns come back through the solver's column scaling; give
            # them their exact values (a fixed Var's value is the fixed value)
            self._set_nonant_x(self._fix_val, self._fixed)
        rec = {"wall_s": None, "t0": t0, "gripe": gripe}
        self.solve_stats.append(rec)
        if total.value == -1:
            self._solve_pending = True
            if getattr(self, "_expect_ahead_wanted", False):
                self._expect_ahead()
        else:
            self._record_solve(rec, int(total.value), 0)
        if self.extensions is not None:
            if _overrides(self.extobject, "post_solve"):
                self._settle()
                stc = self._status.cpu().numpy()
                sgn = 1.0 if self.is_minimizing else -1.0
                objs = (self._obj.cpu().numpy() + self._c0_int) * sgn
                for k, s in enumerate(self.local_subproblems.values()):
                    self.extobject.post_solve(s, SolveResults(int(stc[k]), float(objs[k])))
            self.extobject.post_solve_loop()
        if dtiming:
            allt = self.mpicomm.gather(self.solve_stats[-1]["wall_s"])
            if self.cylinder_rank == 0:
                print("Batched solve times (seconds): min=%4.2f mean=%4.2f max=%4.2f"
                      % (min(allt), sum(allt) / len(allt), max(allt)))

    def _record_solve(self, rec, total, stragglers):
        lib = self._native
        stt = _native.SolveStats()
        ctx = getattr(self, "_solve_ctx", None) or self._ctx
        lib.check(ctx, lib.last_solve_stats(ctx, ctypes.byref(stt)), "last_solve_stats")
        n_bad = int(stt.not_optimal) + int(stt.infeasible)
        t0, gripe = rec.pop("t0"), rec.pop("gripe")
        rec.update({"pdhg_iters": total, "pdhg_ms": stt.pdhg_ms, "launches": stt.pdhg_launches,
                    "lane_iters": stt.lane_iters, "polish_ms": stt.polish_ms, "ipm_ms": stt.ipm_ms,
                    "lane_ms": stt.lane_ms, "lane_warm_ms": stt.lane_warm_ms,
                    "lane_warm_list_ms": stt.lane_warm_list_ms, "lane_certified": stt.lane_certified,
                    "lane_warm_certified": stt.lane_warm_certified,
                    "lane_first_certified": stt.lane_first_certified, "stragglers": stragglers,
                    "wg_certified": stt.wg_certified, "wg_ms": stt.wg_ms,
                    "sp_certified": stt.sp_certified, "sp_warm_rounds": stt.sp_warm_rounds,
                    "sp_ipm_its": stt.sp_ipm_its, "sp_cold_rounds": stt.sp_cold_rounds,
                    "sp_refine": stt.sp_refine, "sp_ms": stt.sp_ms,
                    "wall_s": time.perf_counter() - t0, "not_optimal": int(stt.not_optimal),
                    "infeasible": int(stt.infeasible)})
        if n_bad and gripe:
            stc = self._status.cpu().numpy()
            name = self.__class__.__name__
            if self.spcomm:
                name = self.spcomm.__class__.__name__
            for k in np.nonzero(stc != OPTIMAL)[0][:10]:
                print("[%s] Solve failed for scenario %s" % (name, self.local_scenario_names[k]))
                print("status=", {ITER_LIMIT: "iteration limit", NUMERIC_FAIL: "numerical failure",
                                  INFEASIBLE: "infeasible"}.get(int(stc[k]), int(stc[k])))

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
        if getattr(self, "_iter0_deferred", False):
            self._resolve_deferred_iter0()
        if self._solve_pending or getattr(self, "_w_uncommitted", False):
            self._settle_pending()

    def _settle_pending(self):
        self._sync_solve()

    # ------------------------------------------------------------ expectations
    def _expect(self, values):
        """[sum p*values, sum p, sum p*[optimal]] over the local scenarios (device);
        cached until the next device operation (Iter0 asks three times: E1,
        feas_prob, Ebound)."""
        self._settle()
        key = (values.data_ptr(), self._host_epoch)
        if getattr(self, "_expect_key", None) == key:
            return self._expect_buf
        lib = self._native
        lib.check(self._ctx, lib.expect(self._ctx, self._prob.data_ptr(), values.data_ptr(),
                                        self._status.data_ptr(), self._expect_buf.data_ptr(),
                                        self._stream()), "expect")
        self._expect_key = key
        return self._expect_buf

    def Eobjective(self, verbose=False):
        """sum_s p_s * objective_s incl. active W/prox terms (spopt.py:310-343)."""
        self._objective_now()
        buf = self._expect(self._obj_eval).clone()
        g = self.mpicomm.allreduce_(buf[0:1] + self._pc0)
        v = float(g.item())
        return v if self.is_minimizing else -v

    def _objective_now(self):
        """Objective of the current x under the current W/xbar/rho and W_on/prox_on."""
        self._settle()
        if not hasattr(self, "_obj_eval"):
            self._obj_eval = torch.zeros_like(self._obj)
        if self._prox_lin is not None:
            self._prox_lin.objective_into(self._obj_eval)
            self._bump()
            return
        self._set_ph_terms()
        lib = self._native
        lib.check(self._ctx, lib.objective(self._ctx, self._x.data_ptr(), self._obj_eval.data_ptr(),
                                           self._stream()), "objective")
        self._bump()

    def _expect_ahead(self):
        """Iter0 (one rank): the expectations of the deferred solve's outputs
        enqueued right behind it, with their copy into a pinned buffer, so that
        E1 / feas_prob / Ebound read them with the solve's own wait instead of
        a second device round trip.  Valid only if finishing the solve changes
        no output (no scenario needed the generic path: the host epoch is
        unchanged); _expect_sums checks that and recomputes otherwise."""
        self._expect_ahead_state = None
        if self.n_proc != 1 or self.device.type != "cuda":
            return
        lib = self._native
        lib.check(self._ctx, lib.expect(self._ctx, self._prob.data_ptr(), self._outer.data_ptr(),
                                        self._status.data_ptr(), self._expect_buf.data_ptr(),
                                        self._stream()), "expect")
        pin = self._pinned_small()
        pin[:3].copy_(self._expect_buf[:3], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._expect_ahead_state = (self._host_epoch, ev)

    def _expect_sums(self):
        """[sum p*outer, sum p, sum p*[optimal]] over ALL ranks, on the host:
        one all-reduce and one device->host copy per solve (Iter0's E1,
        feas_prob and Ebound read the same three numbers)."""
        ahead = getattr(self, "_expect_ahead_state", None)
        if ahead is not None:
            self._expect_ahead_state = None
            self._settle()
            epoch, ev = ahead
            if epoch == self._host_epoch:
                ev.synchronize()
                self._expect_key = (self._outer.data_ptr(), self._host_epoch)   # _expect_buf holds them
                self._expect_sums_val = self._pinned_small()[:3].numpy().copy()
                self._expect_sums_key = self._expect_key
                return self._expect_sums_val
        buf = self._expect(self._outer)
        key = self._expect_key
        if getattr(self, "_expect_sums_key", None) != key:
            R, r = self.n_proc, self.cylinder_rank
            v = self._sums_over_ranks(buf)
            self._expect_sums_val = v
            self._expect_sums_key = key
        return self._expect_sums_val

    def _sums_over_ranks(self, buf):
        """The three expectation sums of buf[:3] over all ranks, on the host."""
        R, r = self.n_proc, self.cylinder_rank
        if R == 1:
            return self._read_small(buf[:3])
        # every rank's three sums side by side (x + 0 is exact), then summed in
        # rank order on the host: the three totals see the same order, so
        # E1 == E_feas exactly when every scenario is feasible (a ring all-reduce
        # orders each element differently)
        t = torch.zeros(3 * R, dtype=torch.float64, device=self.device)
        t[3 * r:3 * r + 3] = buf[:3]
        self.mpicomm.allreduce_(t)
        parts = t.cpu().numpy().reshape(R, 3)
        v = parts[0].copy()
        for q in range(1, R):
            v = v + parts[q]
        return v

    def _pc0_all(self):
        """sum over ranks of the local sum p * objective constant (once)."""
        if getattr(self, "_pc0_sum", None) is None:
            self._pc0_sum = float(self.mpicomm.allreduce_np([self._pc0])[0])
        return self._pc0_sum

    def Ebound(self, verbose=False, extra_sum_terms=None):
        """sum_s p_s * outer_bound_s (+ extra terms), spopt.py:346-391."""
        v = float(self._expect_sums()[0]) + self._pc0_all()
        sgn = 1.0 if self.is_minimizing else -1.0
        if extra_sum_terms is None:
            return sgn * v
        extra = self.mpicomm.allreduce_np(np.asarray(list(extra_sum_terms), dtype=np.float64))
        return sgn * v, extra

    def _update_E1(self):
        self.E1 = float(self._expect_sums()[1])

    def feas_prob(self):
        return float(self._expect_sums()[2])

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

    # ------------------------------------------------------------ nonant fixing
    # spopt.py:536-742.  A fixed nonant is a column with lb = ub = value (what a
    # persistent solver's update_var does); fixedness and values live on the
    # host as [S_local][N] arrays (the reference's per-scenario caches, same
    # slot order), and the solve sees them through phx_set_bounds, uploaded
    # only when fixedness changed.  Nothing is fixed originally (creators
    # express fixed data as bounds).
    def _fix_arrays(self):
        if getattr(self, "_fixed", None) is None:
            S, N = self._S, self.batch.nonant.N
            self._fixed = np.zeros((S, N), dtype=bool)
            self._fix_val = np.zeros((S, N))
            self._fix_dirty = False
        return self._fixed, self._fix_val

    def _nonant_x(self):
        """(S_local, N) current nonant values (host copy)."""
        return self.nonant_values()

    def _set_nonant_x(self, vals, mask=None):
        """Write nonant values (S_local, N) into x on the device (where mask)."""
        self._settle()
        self._x_touched = True
        nn = self.batch.nonant
        S = self._S
        cols = torch.as_tensor(nn.slot_col.astype(np.int64), device=self.device)
        xv = self._x.view(-1, S)
        new = torch.as_tensor(np.ascontiguousarray(np.asarray(vals, dtype=np.float64).T), device=self.device)
        if mask is not None:
            m = torch.as_tensor(np.ascontiguousarray(np.asarray(mask, dtype=bool).T), device=self.device)
            new = torch.where(m, new, xv[cols])
        xv[cols] = new
        self._bump()

    def _cache_by_slot(self, cache, stage_max=None, root_only=False):
        """Per (scenario, slot) values from an ndn-keyed cache, with the
        reference's errors (spopt.py:569-583); returns (vals, mask)."""
        nn = self.batch.nonant
        S, N = self._S, nn.N
        vals = np.zeros((S, N))
        mask = np.zeros((S, N), dtype=bool)
        nlen_of = {}
        for t in range(nn.nstages):
            nlen_of[t] = nn.nlen(t)
        for t in range(nn.nstages):
            if root_only and t > 0:
                break
            if stage_max is not None and t + 1 > stage_max:
                break
            slots = np.nonzero(nn.slot_stage == t + 1)[0]
            names = nn.node_names[t] if not root_only else None
            groups = {"ROOT": np.arange(S)} if names is None else {}
            if names is not None:
                arr = np.asarray(names)
                for nd in dict.fromkeys(names):
                    groups[nd] = np.nonzero(arr == nd)[0]
            for nd, ss in groups.items():
                if root_only:
                    c = cache
                    if c is None:
                        raise RuntimeError("Empty root cache for scen={}".format(self.local_scenario_names[0]))
                    if len(c) != nlen_of[0]:
                        raise RuntimeError("Needed {} nonant Vars for 'ROOT', got {}".format(nlen_of[0], len(c)))
                else:
                    if nd not in cache:
                        raise RuntimeError("Could not find {} in {}".format(nd, cache))
                    c = cache[nd]
                    if c is None:
                        raise RuntimeError("Empty cache for scen={}, node={}"
                                           .format(self.local_scenario_names[int(ss[0])], nd))
                    if len(c) != nlen_of[t]:
                        raise RuntimeError("Needed {} nonant Vars for {}, got {}".format(nlen_of[t], nd, len(c)))
                c = np.asarray(c, dtype=np.float64)
                for j in slots:
                    vals[ss, j] = c[nn.slot_local[j]]
                    mask[ss, j] = True
        return vals, mask

    def _fix_where(self, vals, mask):
        fixed, fv = self._fix_arrays()
        fixed |= mask
        fv[mask] = vals[mask]
        self._fix_dirty = True
        self._set_nonant_x(vals, mask)

    def _fix_nonants(self, cache):
        """Fix every local scenario's nonants at ``cache[ndn][i]`` (spopt.py:557-591)."""
        vals, mask = self._cache_by_slot(cache)
        self._fix_where(vals, mask)

    def _fix_root_nonants(self, root_cache):
        """Fix the ROOT nonants at ``root_cache[i]`` (spopt.py:593-636)."""
        if "ROOT" not in self.all_nodenames:
            raise RuntimeError("Could not find a 'ROOT' node in scen {}".format(self.local_scenario_names[0]))
        vals, mask = self._cache_by_slot(root_cache, root_only=True)
        self._fix_where(vals, mask)

    def _save_nonants(self):
        """nonant_cache / fixedness_cache <- current values and fixedness (spopt.py:665-687)."""
        fixed, _ = self._fix_arrays()
        self.nonant_cache = np.ascontiguousarray(self._nonant_x())
        self.fixedness_cache = fixed.copy()

    def _put_nonant_cache(self, cache):
        """Flat scenario-major values into nonant_cache (spopt.py:530-543)."""
        if getattr(self, "nonant_cache", None) is None:
            raise RuntimeError("Rank {} Scenario {} nonant_cache is None (call _save_nonants first?)"
                               .format(self.global_rank, self.local_scenario_names[0]))
        S, N = self.nonant_cache.shape
        assert len(cache) >= S * N
        self.nonant_cache[:] = np.asarray(cache[:S * N], dtype=np.float64).reshape(S, N)

    def _restore_nonants(self):
        """Values and fixedness back from nonant_cache / fixedness_cache (spopt.py:638-662)."""
        fixed, fv = self._fix_arrays()
        fixed[:] = self.fixedness_cache
        fv[:] = self.nonant_cache
        self._fix_dirty = True
        self._set_nonant_x(self.nonant_cache)

    def _save_original_nonants(self):
        """original_nonants / original_fixedness (spopt.py:690-710).  The values are
        kept as a device copy (one gather into a buffer allocated with the
        problem: no allocation and no host round trip inside Iter0);
        ``original_nonants`` reads them back on first use, and fixedness is
        copied only when something was ever fixed."""
        self._settle()
        S = self._S
        if getattr(self, "_x_touched", True):
            torch.index_select(self._x.view(-1, S), 0, self._slot_cols_dev, out=self._orig_nonants_dev)
        # (else x still holds its initial zeros, as _orig_nonants_dev does: nothing to copy)
        self._orig_nonants_saved = True
        self._orig_nonants_host = None
        fixed = getattr(self, "_fixed", None)
        self._orig_fixed = None if fixed is None else fixed.copy()   # None: nothing fixed
        self._orig_fixed_saved = True

    @property
    def original_nonants(self):
        if getattr(self, "_orig_nonants_host", None) is None:
            if not getattr(self, "_orig_nonants_saved", False):
                raise AttributeError("original_nonants: _save_original_nonants has not run")
            self._orig_nonants_host = np.ascontiguousarray(self._orig_nonants_dev.cpu().numpy().T)
        return self._orig_nonants_host

    @original_nonants.setter
    def original_nonants(self, vals):
        self._orig_nonants_host = np.ascontiguousarray(np.asarray(vals, dtype=np.float64))
        self._orig_nonants_saved = True

    @property
    def original_fixedness(self):
        if not getattr(self, "_orig_fixed_saved", False):
            return None
        if self._orig_fixed is None:
            self._orig_fixed = np.zeros((self._S, self.batch.nonant.N), dtype=bool)
        return self._orig_fixed

    @original_fixedness.setter
    def original_fixedness(self, vals):
        self._orig_fixed = None if vals is None else np.asarray(vals, dtype=bool).copy()
        self._orig_fixed_saved = vals is not None

    def _restore_original_nonants(self):
        """spopt.py:713-741."""
        fixed, fv = self._fix_arrays()
        orig_fixed = getattr(self, "original_fixedness", None)
        fixed[:] = False if orig_fixed is None else orig_fixed
        fv[:] = self.original_nonants
        self._fix_dirty = True
        self._set_nonant_x(self.original_nonants)

    def _restore_original_fixedness(self):
        """Original fixedness, current values (spopt.py:546-554)."""
        fixed, fv = self._fix_arrays()
        orig = getattr(self, "original_fixedness", None)
        new = np.zeros_like(fixed) if orig is None else orig
        if not np.array_equal(new, fixed):
            fv[:] = self._nonant_x()
            fixed[:] = new
            self._fix_dirty = True

    def _unfix_nonants(self):
        fixed, _ = self._fix_arrays()
        if fixed.any():
            fixed[:] = False
            self._fix_dirty = True

    def _apply_fixing(self):
        """Upload per-scenario bounds with the fixed nonants (phx_set_bounds),
        or restore the model's bounds when nothing is fixed."""
        if not getattr(self, "_fix_dirty", False):
            return
        lib = self._native
        fixed = self._fixed
        if not fixed.any():
            lib.check(self._ctx, lib.set_bounds(self._ctx, None, None, self._stream()), "set_bounds")
            self._fix_lb = self._fix_ub = None
        else:
            if self._bundles is not None:
                raise NotImplementedError("fixing nonants of bundled scenarios (bundles_per_rank) is not supported")
            b = self.batch
            n, S = b.n, self._S
            cols = torch.as_tensor(b.nonant.slot_col.astype(np.int64), device=self.device)
            lb = self._dev["lb"].view(n, -1).expand(n, S).contiguous()
            ub = self._dev["ub"].view(n, -1).expand(n, S).contiguous()
            m = torch.as_tensor(np.ascontiguousarray(fixed.T), device=self.device)
            v = torch.as_tensor(np.ascontiguousarray(self._fix_val.T), device=self.device)
            lb[cols] = torch.where(m, v, lb[cols])
            ub[cols] = torch.where(m, v, ub[cols])
            lib.check(self._ctx, lib.set_bounds(self._ctx, lb.data_ptr(), ub.data_ptr(), self._stream()),
                      "set_bounds")
            self._fix_lb, self._fix_ub = lb, ub
        self._fix_dirty = False
