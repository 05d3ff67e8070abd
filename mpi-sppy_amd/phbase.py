"""PHBase — the PH iterate on the GPU behind the reference API.

Mirrors ``mpisppy.phbase.PHBase`` (``mpisppy/phbase.py:176-1050``): same
constructor and options contract (``options_check`` 726-755), same
``Compute_Xbar`` -> ``Update_W`` -> ``convergence_diff`` -> stop test ->
``solve_loop`` order (``iterk_loop`` 875-979), same ``Iter0`` checks
(E1 / feasibility ``quit()``, 812-823), hooks (``pre_iter0``, ``post_iter0``,
``post_iter0_after_sync``, ``miditer``, ``enditer``, ``enditer_after_sync``,
``post_everything``), converger and hub (``spcomm.sync`` / ``is_converged``).

Device mapping:
  Compute_Xbar      phx_xbar (segmented per-node reduction) + ONE allreduce
                    of the fused [sum p x | sum p x^2] buffer (RCCL on GPU)
  Update_W          phx_update_w (W += rho (x - xbar), |x - xbar| per scenario,
                    per-emulated-rank segment sums)
  convergence_diff  allreduce of the per-rank sums; mean of per-rank means
                    (phbase.py:330-343)
  solve_loop        phx_set_ph_terms + phx_solve (batched PDHG + KKT polish)
"""
import ctypes
import math
import time

import numpy as np
import torch

from . import _native
from .spopt import SPOpt
from .spbase import _global_toc


class PHBase(SPOpt):
    def __init__(self, options, all_scenario_names, scenario_creator, scenario_denouement=None,
                 all_nodenames=None, mpicomm=None, scenario_creator_kwargs=None, extensions=None,
                 extension_kwargs=None, ph_converger=None, rho_setter=None, variable_probability=None,
                 _native_lib=None, _device=None):
        super().__init__(options, all_scenario_names, scenario_creator,
                         scenario_denouement=scenario_denouement, all_nodenames=all_nodenames,
                         mpicomm=mpicomm, extensions=extensions, extension_kwargs=extension_kwargs,
                         scenario_creator_kwargs=scenario_creator_kwargs,
                         variable_probability=variable_probability,
                         _native_lib=_native_lib, _device=_device)
        self.options = options
        self.options_check()
        self.ph_converger = ph_converger
        self.rho_setter = rho_setter
        self.iter0_solver_options = options["iter0_solver_options"]
        self.iterk_solver_options = options["iterk_solver_options"]
        self.current_solver_options = self.iter0_solver_options
        self.convobject = None
        self.conv = None
        self._PHIter = 0
        self.attach_xbars()
        # the device loop's buffers and events, allocated with the problem
        # (phx_iterk_prepare) so no PH iteration pays an allocation
        self._native_comm = False
        # the device loop's solver tier is decided from each rank's own problem;
        # the ranks must agree (min over the cylinder) before anything
        # collective depends on it -- the RCCL setup below, phx_iterk's
        # per-iteration all-reduce -- or ranks that chose differently would wait
        # on each other forever
        self._loop_veto = False
        local = (self.batch.nonant.N > 0 and self.NNS > 0
                 and self._device_loop_solver(self._solve_opts(self.iterk_solver_options)))
        agreed = local
        if self.n_proc > 1:
            agreed = bool(self.mpicomm.allreduce_np(np.array([1 if local else 0], dtype=np.int64), op="min")[0])
        self._loop_veto = local and not agreed
        if agreed:
            if self._want_native_comm():
                self._setup_native_comm()
            lib = self._native
            lib.check(self._ctx, lib.iterk_prepare(self._ctx, ctypes.byref(self._iterk_argstruct())),
                      "iterk_prepare")

    # ------------------------------------------------------------ state
    def attach_xbars(self):
        """xbar/xsqbar per (node, slot) live on the device (phbase.py:1040-1050)."""
        self._xbar_node.zero_()
        self._xsqbar_node.zero_()

    def attach_Ws_and_prox(self):
        """W = 0, rho = defaultPHrho, W_on = prox_on = 0 (phbase.py:585-602)."""
        N, S = self.batch.nonant.N, self._S
        self._W = torch.zeros(max(N, 1) * S, dtype=torch.float64, device=self.device)
        # second W buffer: an Update_W issued while a deferred solve may still
        # owe some scenarios (stragglers) writes here and is committed by
        # convergence_diff once the solve is known final (see _settle)
        self._W_alt = torch.zeros_like(self._W)
        self._w_uncommitted = False
        self._rho = torch.full((max(N, 1) * S,), float(self.options["defaultPHrho"]),
                               dtype=torch.float64, device=self.device)
        self.W_on = 0
        self.prox_on = 0

    def attach_PH_to_objective(self, add_duals, add_prox):
        """The PH terms are applied by the native solver (phx_set_ph_terms);
        with ``linearize_proximal_terms`` the prox term's x^2 is replaced by
        tangent cuts (phbase.py:628-692; prox_approx.py)."""
        self._attach_duals = bool(add_duals)
        self._attach_prox = bool(add_prox)
        if add_prox and self.options.get("linearize_proximal_terms", False) and self.batch.nonant.N:
            from .prox_approx import ProxLinSolver
            if self._bundles is not None:
                raise NotImplementedError("linearize_proximal_terms with bundles_per_rank is not supported")
            self._prox_lin = ProxLinSolver(self, self.options.get("proximal_linearization_tolerance", 1.e-1),
                                           self.options.get("initial_proximal_cut_count", 2))

    def PH_Prep(self, attach_duals=True, attach_prox=True):
        self.attach_Ws_and_prox()
        self.attach_PH_to_objective(attach_duals, attach_prox)

    def options_check(self):
        required = ["solver_name", "PHIterLimit", "defaultPHrho", "convthresh", "verbose", "display_progress"]
        self._options_check(required, self.options)
        if "display_timing" not in self.options:
            self.options["display_timing"] = False
        if "display_convergence_detail" not in self.options:
            self.options["display_convergence_detail"] = False

    # ------------------------------------------------------------ PH pieces
    def Compute_Xbar(self, verbose=False):
        """Per-node sum_s prob_coeff * x and * x^2, allreduced (phbase.py:27-107)."""
        lib = self._native
        lib.check(self._ctx, lib.xbar(self._ctx, self._tree, self._x.data_ptr(), self._pc.data_ptr(),
                                      self._partial.data_ptr(), self._node_buf.data_ptr(), self._stream()),
                  "xbar")
        self.mpicomm.allreduce_(self._node_buf)
        self._conv_cache = None
        self._bump()
        if verbose and self.cylinder_rank == 0:
            print("xbar:", self._xbar_node.cpu().numpy())

    def _update_w_and_diff(self, update):
        lib = self._native
        W_out = self._W
        if update and self._solve_pending:
            W_out = self._W_alt                  # out of place until the solve is known final
            self._w_uncommitted = True
        lib.check(self._ctx, lib.update_w(self._ctx, self._x.data_ptr(), self._xbar_node.data_ptr(),
                                          self._xbar_idx_t.data_ptr(), self._rho.data_ptr(),
                                          self._W.data_ptr(), W_out.data_ptr(), int(update), None,
                                          self._conv_R, self._seg_s0, self._seg_s1,
                                          self._seg_sums.data_ptr(), self._stream()), "update_w")
        if update and self._prob0_mask_t is not None:
            W_out.mul_(self._prob0_mask_t)     # zero-probability slots keep W = 0 (phbase.py:314-318)
        self._conv_cache = self._seg_sums      # consumed (all-reduced) by convergence_diff
        self._conv_value = None
        self._conv_updated_w = bool(update)
        self._bump()

    def _settle_pending(self):
        """Finish a deferred solve; an optimistic Update_W issued behind it is
        committed, or redone in place if some scenario's x changed (collective
        over ranks when such an update is outstanding)."""
        n = self._sync_solve()
        if self._w_uncommitted:
            if self.n_proc > 1:
                t = torch.tensor([float(n)], dtype=torch.float64, device=self.device)
                self.mpicomm.allreduce_(t)
                n = int(t.item())
            self._w_uncommitted = False
            if n > 0:
                self.Compute_Xbar(False)
                self._update_w_and_diff(self._conv_updated_w)
            else:
                self._W, self._W_alt = self._W_alt, self._W

    def Update_W(self, verbose):
        """W += rho (x - xbar) (phbase.py:293-318)."""
        self._update_w_and_diff(True)
        if verbose and self.cylinder_rank == 0:
            print("W:", self._W.view(-1, self._S)[:, :3].cpu().numpy())

    def convergence_diff(self):
        """(1/R) sum_r mean_{(s,i) in rank r} |x - xbar|  (phbase.py:321-343)."""
        if getattr(self, "_conv_cache", None) is None:
            self._update_w_and_diff(False)
        if getattr(self, "_conv_value", None) is None:
            R = self._conv_R
            t = self._conv_cache
            pending = self._solve_pending
            redo = False
            single = self.n_proc == 1 and self.device.type == "cuda"
            if single:
                # read the sums back asynchronously into pinned memory; the wait
                # below covers it (one host synchronisation per PH step)
                if getattr(self, "_conv_host", None) is None:
                    self._conv_host = torch.empty(R + 1, dtype=torch.float64, pin_memory=True)
                    self._conv_evt = torch.cuda.Event()
                self._conv_host.copy_(t, non_blocking=True)
                self._conv_evt.record()
            if pending:
                # Deferred solve: Compute_Xbar / Update_W were enqueued behind it
                # optimistically.  Finish it now (the GPU is busy with them) and
                # count, over all ranks, the scenarios it had to hand to the
                # generic path: their x was not final when x-bar was formed.
                n_local = self._sync_solve()
                if self.n_proc > 1:
                    t[R].fill_(float(n_local))
                else:
                    redo = n_local > 0
            if single and not redo:
                self._conv_evt.synchronize()
                v = self._conv_host.numpy()
            else:
                self.mpicomm.allreduce_(t)
                v = t.cpu().numpy()
            if pending and (redo or (self.n_proc > 1 and v[R] > 0)):
                # redo the step on the now final x; W from the committed buffer,
                # updated in place (the optimistic W_alt is discarded)
                self._w_uncommitted = False
                upd = self._conv_updated_w
                self.Compute_Xbar(False)
                self._update_w_and_diff(upd)
                t = self._conv_cache
                if self.n_proc > 1:
                    t[R].fill_(0.0)
                self.mpicomm.allreduce_(t)
                v = t.cpu().numpy()
            if self._w_uncommitted:
                self._W, self._W_alt = self._W_alt, self._W
                self._w_uncommitted = False
            cnt = self._conv_counts
            tot = 0.0
            for r in range(R):
                if cnt[r] > 0:
                    tot += v[r] / cnt[r]
            self._conv_value = tot / R
        return self._conv_value

    def _populate_W_cache(self, cache, padding):
        """Flat scenario-major W export (phbase.py:346-366)."""
        self._settle()
        N, S = self.batch.nonant.N, self._S
        if len(cache) - padding < N * S:
            raise RuntimeError("W cache length mismatch detected by %s that has total W len %d but "
                               "passed cache len-1=%d; len(nonants)=%d"
                               % (self.__class__.__name__, N * S, len(cache) - 1, N))
        flat = self._W.view(N, S).t().contiguous().view(-1).cpu().numpy()
        cache[:N * S] = flat
        assert N * S == len(cache) - padding

    def W_from_flat_list(self, flat_list):
        """Set W from a flat scenario-major list (phbase.py:369-385)."""
        self._settle()
        N, S = self.batch.nonant.N, self._S
        a = torch.as_tensor(np.asarray(flat_list[:N * S], dtype=np.float64)).view(S, N).t().contiguous()
        self._W.copy_(a.view(-1).to(self.device))
        self._bump()

    def _use_rho_setter(self, verbose):
        """rho from a user callback returning [(id(var), rho)] (phbase.py:387-406)."""
        if self.rho_setter is None:
            return
        kw = self.options.get("rho_setter_kwargs", {})
        didit = 0
        for sname, view in self.local_scenarios.items():
            target = self._models[sname] if self._models is not None else view
            for vid, rho in self.rho_setter(target, **kw):
                j = view._slot_of_varid(vid)
                self._host_write("rho", j, view._s, rho)
                didit += 1
        if verbose and self.cylinder_rank == 0:
            print("rho_setter set", didit)

    def _disable_prox(self):
        self.prox_on = 0

    def _disable_W(self):
        self.W_on = 0

    def disable_W_and_prox(self):
        self._disable_W()
        self._disable_prox()

    def _reenable_prox(self):
        self.prox_on = 1 if getattr(self, "_attach_prox", True) else 0

    def _reenable_W(self):
        self.W_on = 1 if getattr(self, "_attach_duals", True) else 0

    def reenable_W_and_prox(self):
        self._reenable_W()
        self._reenable_prox()

    @property
    def W_disabled(self):
        return not bool(self.W_on)

    @property
    def prox_disabled(self):
        return not bool(self.prox_on)

    def post_solve_bound(self, solver_options=None, verbose=False):
        """Lagrangian bound with the current W (phbase.py:443-491)."""
        if self.cylinder_rank == 0:
            print("Warning: Lagrangian bounds might not be correct in certain cases where there are "
                  "integers not subject to non-anticipativity and those integers do not reach integrality.")
        if self.W_disabled:
            self._reenable_W()
        self._disable_prox()
        # fixed variables can lead to an invalid lower bound
        self._restore_original_fixedness()
        self.solve_loop(solver_options=solver_options, dis_prox=False, gripe=True, tee=False, verbose=verbose)
        bound = self.Ebound(verbose)
        self._reenable_prox()
        if verbose and self.cylinder_rank == 0:
            print("Post-solve Lagrangian bound: %.4f" % bound)
        return bound

    def solve_loop(self, solver_options=None, use_scenarios_not_subproblems=False, dtiming=False,
                   dis_W=False, dis_prox=False, gripe=False, disable_pyomo_signal_handling=False,
                   tee=False, verbose=False):
        """W/prox toggles around the batched solve (phbase.py:494-568)."""
        if dis_W and dis_prox:
            self.disable_W_and_prox()
        elif dis_W:
            self._disable_W()
        elif dis_prox:
            self._disable_prox()
        super().solve_loop(solver_options, use_scenarios_not_subproblems, dtiming, gripe,
                           disable_pyomo_signal_handling, tee, verbose)
        if dis_W and dis_prox:
            self.reenable_W_and_prox()
        elif dis_W:
            self._reenable_W()
        elif dis_prox:
            self._reenable_prox()

    # ------------------------------------------------------------ loops
    def _can_defer_iter0(self):
        """Iter0's checks (E1, feasibility, trivial bound) may wait for the device
        loop: ph_main asked for it, nothing observes the state between Iter0 and
        the first iteration (no hooks, converger, hub, rho setter, printouts), and
        the iterations will run in phx_iterk, which then adopts Iter0's deferred
        solve (no host round trip between them)."""
        if not getattr(self, "_defer_iter0_checks", False):
            return False
        if (self.extensions is not None or self.ph_converger is not None or self.spcomm is not None
                or self.rho_setter is not None):
            return False
        o = self.options
        if o["display_progress"] or o["verbose"] or o["display_convergence_detail"] or o["display_timing"]:
            return False
        if int(o["PHIterLimit"]) < 1:
            return False
        # a total probability Iter0's check would reject quits before any PH
        # iteration (phbase.py:812-817): checked here, so a deferred Iter0
        # never runs iterations first (the same sum the device computes; the
        # tolerance is far above their rounding difference)
        # (host data, once per probability array: no device read in the timed
        # Iter0; both caches hold the array they summed and compare with `is`)
        pre_E1 = getattr(self, "_E1_pre", None)
        if pre_E1 is not None and pre_E1[0] is self.batch.prob:
            E1 = pre_E1[1]
        else:
            pre = getattr(self, "_prob_local_sum", None)
            if pre is not None and pre[0] is self.batch.prob:
                E1 = pre[1]   # (summed at construction, spbase._look_and_leap)
            else:
                E1 = float(np.sum(np.asarray(self.batch.prob, dtype=np.float64)))
            if self.n_proc > 1:
                E1 = float(self.mpicomm.allreduce_np(np.array([E1]), op="sum")[0])
            self._E1_pre = (self.batch.prob, E1)
        if abs(1 - E1) > self.E1_tolerance:
            return False
        saved = self.current_solver_options
        self.current_solver_options = self.options["iterk_solver_options"]
        try:
            return self._native_loop_ok()
        finally:
            self.current_solver_options = saved

    def _iter0_checks(self, v):
        """phbase.py:805-856 on the sums [sum p obj, sum p, sum p [optimal]] of
        Iter0's solve: E1 and feasibility (quit() on failure), trivial bound."""
        self.E1 = float(v[1])
        if abs(1 - self.E1) > self.E1_tolerance:
            if self.cylinder_rank == 0:
                print("ERROR")
                print("Total probability of scenarios was ", self.E1)
                print("E1_tolerance = ", self.E1_tolerance)
            quit()
        feasP = float(v[2])
        if feasP != self.E1:
            if self.cylinder_rank == 0:
                print("ERROR")
                print("Infeasibility detected; E_feas, E1=", feasP, self.E1)
            quit()
        sgn = 1.0 if self.is_minimizing else -1.0
        self.trivial_bound = sgn * (float(v[0]) + self._pc0_all())

    def _resolve_deferred_iter0(self, device_sums=False):
        """The deferred Iter0 checks, on Iter0's objectives / statuses (copied by
        phx_iterk when it adopted the solve, else by Iter0 or here).
        device_sums: phx_iterk already evaluated the expectations of the adopted
        solve into _expect_buf and its pinned host copy (iter0_expect_host)."""
        self._iter0_deferred = False
        if device_sums:
            self._expect_key = None
            if self.n_proc == 1:
                self._iter0_checks(self._iter0_exp_host.tolist())
            else:
                self._iter0_checks(self._sums_over_ranks(self._expect_buf))
            return
        if self._solve_pending:
            # not adopted (the loop did not run on the device): finish it here,
            # before anything else touches its outputs
            self._sync_solve()
            self._iter0_obj_dev.copy_(self._obj)
            self._iter0_status_dev.copy_(self._status)
        lib = self._native
        lib.check(self._ctx, lib.expect(self._ctx, self._prob.data_ptr(), self._iter0_obj_dev.data_ptr(),
                                        self._iter0_status_dev.data_ptr(), self._expect_buf.data_ptr(),
                                        self._stream()), "expect")
        self._expect_key = None
        self._iter0_checks(self._sums_over_ranks(self._expect_buf))

    def Iter0(self):
        """phbase.py:758-872.  Returns the trivial bound, or None when ph_main
        deferred Iter0's checks to the device loop (_can_defer_iter0): they run
        right after it, before anything reads the state (ph_main returns
        self.trivial_bound then)."""
        self._check_stream()
        if self._can_defer_iter0():
            return self._iter0_deferred_start()
        if self.extensions is not None:
            self.extobject.pre_iter0()
        # fixedness / values as the extensions left them (phbase.py:788): what
        # post_solve_bound restores (_restore_original_fixedness)
        self._save_original_nonants()
        verbose = self.options["verbose"]
        dprogress = self.options["display_progress"]
        dtiming = self.options["display_timing"]
        have_extensions = self.extensions is not None
        have_converger = self.ph_converger is not None
        self._PHIter = 0
        self._create_solvers()
        teeme = bool(self.options.get("tee-rank0-solves", False)) and self.cylinder_rank == 0
        # E1 / feas_prob / Ebound read their sums behind the solve's own wait
        # (SPOpt._expect_ahead)
        self._expect_ahead_wanted = True
        try:
            self.solve_loop(solver_options=self.current_solver_options, dtiming=dtiming, gripe=True,
                            tee=teeme, verbose=verbose)
        finally:
            self._expect_ahead_wanted = False
        self._update_E1()
        if abs(1 - self.E1) > self.E1_tolerance:
            if self.cylinder_rank == 0:
                print("ERROR")
                print("Total probability of scenarios was ", self.E1)
                print("E1_tolerance = ", self.E1_tolerance)
            quit()
        feasP = self.feas_prob()
        if feasP != self.E1:
            if self.cylinder_rank == 0:
                print("ERROR")
                print("Infeasibility detected; E_feas, E1=", feasP, self.E1)
            quit()
        if have_extensions:
            self.extobject.post_iter0()
        if self.spcomm is not None:
            self.spcomm.sync()
        if have_extensions:
            self.extobject.post_iter0_after_sync()
        if self.rho_setter is not None:
            self._use_rho_setter(verbose and self.cylinder_rank == 0)
        if have_converger:
            self.convobject = self.ph_converger(self)
        self.conv = None
        self.trivial_bound = self.Ebound(verbose)
        # per-scenario Iter0 optima (the outer bounds the trivial bound sums), on the device
        self._iter0_obj_dev.copy_(self._obj)
        if dprogress and self.cylinder_rank == 0:
            print("")
            print("After PH Iteration", self._PHIter)
            print("Trivial bound =", self.trivial_bound)
            print("PHBase Convergence Metric =", self.conv)
            print("Elapsed time: %6.2f" % (time.perf_counter() - self.start_time))
        if self.options["display_convergence_detail"]:
            self.report_var_values_at_rank0(header="Convergence detail:")
        self.reenable_W_and_prox()
        self.current_solver_options = self.options["iterk_solver_options"]
        return self.trivial_bound

    def _iter0_deferred_start(self):
        """Iter0 without its host synchronisation: the batched LP solve is
        enqueued (deferred); E1 / feasibility / trivial bound are evaluated after
        the device loop, which adopts the solve (phx_iterk)."""
        self._save_original_nonants()
        self._PHIter = 0
        self._create_solvers()
        self.solve_loop(solver_options=self.current_solver_options, gripe=True, tee=False,
                        verbose=self.options["verbose"])
        if not self._solve_pending:
            # already final (nothing left to adopt): Iter0's objectives / statuses now
            self._iter0_obj_dev.copy_(self._obj)
            self._iter0_status_dev.copy_(self._status)
        self._iter0_deferred = True
        self._iter0_was_deferred = True
        self.trivial_bound = None
        self.conv = None
        self.reenable_W_and_prox()
        self.current_solver_options = self.options["iterk_solver_options"]
        return None

    def _native_loop_ok(self):
        """The device-driven loop (phx_iterk) runs the same iterations when no
        per-iteration host hook or printout needs the host between steps."""
        o = self.options
        if self.extensions is not None or self.ph_converger is not None or self.spcomm is not None:
            return False
        if o["display_progress"] or o["verbose"] or o["display_convergence_detail"]:
            return False
        if self._bundles is not None or self._prox_lin is not None:   # (host-driven solves)
            return False
        so = self.current_solver_options or {}
        if not int(so.get("native_loop", 1)):
            return False
        if getattr(self, "_fixed", None) is not None and self._fixed.any():
            return False
        if self._prob0_mask_t is not None:      # W masked after every Update_W: the host loop
            return False
        if self.NNS == 0 or self.batch.nonant.N == 0:
            return False
        return self._device_loop_solver(self._solve_opts(so))

    def _device_loop_solver(self, so):
        """Which solve phx_iterk can run per iteration: the lane solver (jit on),
        or, above its size limits, the workgroup warm pass (k_wg_warm), or above
        those the sparse solver's warm pass (k_sp_solve).  False on every rank
        when some rank of the cylinder cannot (_loop_veto, set at construction)."""
        if getattr(self, "_loop_veto", False):
            return False
        info = getattr(self, "_jit_info", None)
        if info is None:
            info = self._jit_info = self._native.jit_info(self._ctx).decode()
        if info.startswith("on") and int(so.lane_solver):
            return True
        if int(so.polish) <= 0 or int(so.warm_start) <= 0:
            return False
        if "workgroup solver on" in info and int(so.wg_warm) > 0:
            return True
        # above the workgroup limits: the sparse solver's warm pass (netdes)
        return "sparse solver on" in info and int(so.sp) > 0

    def _want_native_comm(self):
        """phx_iterk's per-iteration all-reduce from C (an RCCL communicator of
        the context, phx_set_comm) rather than a Python callback into
        torch.distributed: on GPUs with several ranks over RCCL by default
        (iterk_solver_options {"native_comm": 0} keeps the callback; 2 also
        builds a one-rank communicator, a test hook for the RCCL path)."""
        mode = int((self.iterk_solver_options or {}).get("native_comm", 1))
        if self.device.type != "cuda" or mode == 0:
            return False
        return mode == 2 or (self.n_proc > 1 and self.mpicomm.backend == "nccl")

    def _setup_native_comm(self):
        """Collective over the cylinder's ranks: rank 0 draws an RCCL unique id,
        the communicator broadcasts it, every rank joins (ncclCommInitRank)."""
        lib = self._native
        uid = ctypes.create_string_buffer(128)
        if self.cylinder_rank == 0:
            lib.check(self._ctx, lib.comm_unique_id(uid), "comm_unique_id")
        raw = self.mpicomm.bcast(uid.raw if self.cylinder_rank == 0 else None, root=0)
        uid = ctypes.create_string_buffer(raw, 128)
        lib.check(self._ctx, lib.set_comm(self._ctx, uid, self.n_proc, self.cylinder_rank), "set_comm")
        self._native_comm = True

    def _allreduce_cb(self):
        if getattr(self, "_ar_cb", None) is None:
            bufs = {self._node_stage.data_ptr(): self._node_stage, self._seg_sums.data_ptr(): self._seg_sums}
            comm = self.mpicomm
            dev = self.device
            ext = {}

            def cb(user, ptr, count, stream):
                # the collective is enqueued on phx_iterk's own stream (passed in
                # explicitly), so it orders after the x-bar/segment kernels that
                # produced the buffer and before the kernels that consume it
                try:
                    if dev.type == "cuda" and stream:
                        s = ext.get(stream)
                        if s is None:
                            s = ext[stream] = torch.cuda.ExternalStream(stream, device=dev)
                        # (gloo: Comm.allreduce_ stages through the host -- a blocking
                        # read-back on this stream, the host all-reduce, the result
                        # written back in stream order)
                        with torch.cuda.stream(s):
                            comm.allreduce_(bufs[ptr][:count])
                    else:
                        comm.allreduce_(bufs[ptr][:count])
                    return 0
                except Exception as e:   # reported by phx_iterk as a failed all-reduce
                    print("phx_iterk all-reduce callback failed:", repr(e))
                    return 1
            self._ar_cb = _native.ALLREDUCE_FN(cb)
        return self._ar_cb

    def _iterk_native(self, max_iterations):
        """iterk_loop body on the device (phx_iterk): Compute_Xbar -> Update_W ->
        convergence_diff -> stop test -> solve_loop, pipelined with a device-side
        stop flag (phbase.py:875-979 semantics, same kernels as the host loop).
        A deferred Iter0 solve still pending is adopted by phx_iterk (enqueued
        behind it, no host round trip); Iter0's checks run right after."""
        deferred = getattr(self, "_iter0_deferred", False)
        if not deferred:
            self._settle()
        self._apply_fixing()
        self._set_ph_terms()
        self._x_touched = True
        lib = self._native
        so_dict = self.current_solver_options or {}
        so = self._solve_opts(so_dict)
        so.defer = 0
        a = self._iterk_argstruct()
        a.rho, a.W = self._rho.data_ptr(), self._W.data_ptr()
        a.convthresh = float(self.options["convthresh"])
        a.max_iters = int(max_iterations)
        a.depth = int(so_dict.get("iterk_depth", 4))
        a.timing = int(so_dict.get("iterk_timing", 0))
        # fused mode (one launch per PH iteration, two-stage trees) unless
        # {"iterk_fused": 0}; the library decides whether the problem allows it
        a.node_stage_len = self._node_stage.numel() if int(so_dict.get("iterk_fused", 1)) else 0
        a.iter0_obj = self._iter0_obj_dev.data_ptr() if deferred else None
        a.iter0_status = self._iter0_status_dev.data_ptr() if deferred else None
        if deferred:
            # Iter0's expectations evaluated by phx_iterk behind the adopted solve
            a.iter0_prob, a.iter0_expect = self._prob.data_ptr(), self._expect_buf.data_ptr()
            a.iter0_expect_host = self._iter0_exp_host.data_ptr()
        else:
            a.iter0_prob = a.iter0_expect = a.iter0_expect_host = None
        res = _native.IterkResult()
        t0 = time.perf_counter()
        lib.check(self._ctx, lib.iterk(self._ctx, ctypes.byref(so), ctypes.byref(a), ctypes.byref(res),
                                       self._stream()), "iterk")
        if deferred:
            if res.adopted and self._solve_pending:
                # Iter0's solve, finished inside phx_iterk (phx_last_solve_stats: its statistics)
                # (the host emulation finishes a deferred solve without
                # leftovers at once: recorded then, adopted with none)
                self._solve_pending = False
                self._record_solve(self.solve_stats[-1], 0, int(res.adopted_stragglers))
            self._resolve_deferred_iter0(device_sums=bool(res.adopted))
        return self._iterk_finish(res, time.perf_counter() - t0)

    def _iterk_argstruct(self):
        """phx_iterk_args over this object's device state (built once; W and rho
        are set per call: PH_Prep re-creates them)."""
        a = getattr(self, "_iterk_args", None)
        if a is None:
            a = _native.IterkArgs()
            a.x, a.y, a.obj = self._x.data_ptr(), self._y.data_ptr(), self._obj.data_ptr()
            a.status, a.iters = self._status.data_ptr(), self._iters.data_ptr()
            a.tree = ctypes.pointer(self._tree)
            a.prob_coeff, a.partial = self._pc.data_ptr(), self._partial.data_ptr()
            a.node_sums, a.node_stage = self._node_buf.data_ptr(), self._node_stage.data_ptr()
            a.xbar_idx = self._xbar_idx_t.data_ptr()
            a.nseg = len(self._conv_seg)
            a.seg_s0_host = ctypes.cast(self._seg_s0, ctypes.c_void_p)
            a.seg_s1_host = ctypes.cast(self._seg_s1, ctypes.c_void_p)
            a.seg_sums = self._seg_sums.data_ptr()
            self._conv_counts_c = (ctypes.c_double * len(self._conv_counts))(*self._conv_counts)
            a.conv_counts_host = ctypes.cast(self._conv_counts_c, ctypes.c_void_p)
            a.conv_R = self._conv_R
            if self.n_proc > 1 and not self._native_comm:
                a.allreduce = self._allreduce_cb()
            a.depth = 4
            self._iterk_args = a
        return a

    def _iterk_finish(self, res, wall):
        self._bump()
        self._PHIter = int(res.iters)
        self.conv = float(res.conv) if res.iters > 0 else None
        self._conv_cache = self._seg_sums
        self._conv_value = self.conv
        self._conv_updated_w = True
        self.iter_times = [wall / max(res.iters, 1)] * int(res.iters)
        self.iterk_stats = {"iters": int(res.iters), "converged": bool(res.converged), "solves": int(res.solves),
                            "straggler_stops": int(res.straggler_stops), "stragglers": int(res.stragglers),
                            "not_optimal": int(res.not_optimal), "lane_warm_ms": float(res.warm_ms),
                            "warm_launches": int(res.warm_launches), "wall_s": wall,
                            "fused": bool(res.fused)}
        if res.not_optimal:
            stc = self._status.cpu().numpy()
            name = self.__class__.__name__
            for k in np.nonzero(stc != 1)[0][:10]:
                print("[%s] Solve failed for scenario %s" % (name, self.local_scenario_names[k]))
        return res

    def iterk_loop(self):
        """phbase.py:875-979."""
        self._check_stream()
        verbose = self.options["verbose"]
        have_extensions = self.extensions is not None
        have_converger = self.ph_converger is not None
        dprogress = self.options["display_progress"]
        dtiming = self.options["display_timing"]
        self.conv = None
        max_iterations = int(self.options["PHIterLimit"])
        self.iter_times = []
        if getattr(self, "_iter0_deferred", False) and not self._native_loop_ok():
            self._resolve_deferred_iter0()
        if self._native_loop_ok():
            res = self._iterk_native(max_iterations)
            if not res.converged:
                self.mpicomm.Barrier()
                if self.cylinder_rank == 0 and (dprogress or verbose):
                    _global_toc("Reached user-specified limit=%d on number of PH iterations" % max_iterations)
            return
        for self._PHIter in range(1, max_iterations + 1):
            iteration_start_time = time.time()
            if dprogress and self.cylinder_rank == 0:
                _global_toc("Initiating PH Iteration %d" % self._PHIter)
            self.Compute_Xbar(verbose)
            self.Update_W(verbose)
            self.conv = self.convergence_diff()
            if have_extensions:
                self.extobject.miditer()
            if have_converger:
                if self.convobject.is_converged():
                    if self.cylinder_rank == 0:
                        _global_toc("User-supplied converger determined termination criterion reached")
                    break
            elif self.conv is not None:
                if self.conv < self.options["convthresh"]:
                    if self.cylinder_rank == 0 and (dprogress or verbose):
                        _global_toc("Convergence metric=%f dropped below user-supplied threshold=%f"
                                    % (self.conv, self.options["convthresh"]))
                    break
            teeme = bool(self.options.get("tee-rank0-solves", False)) and self.cylinder_rank == 0
            self.solve_loop(solver_options=self.current_solver_options, dtiming=dtiming, gripe=True,
                            disable_pyomo_signal_handling=False, tee=teeme, verbose=verbose)
            if have_extensions:
                self.extobject.enditer()
            if self.spcomm is not None:
                self.spcomm.sync()
                if self.spcomm.is_converged():
                    if self.cylinder_rank == 0:
                        _global_toc("Cylinder convergence")
                    break
            if have_extensions:
                self.extobject.enditer_after_sync()
            self.iter_times.append(time.time() - iteration_start_time)
            if dprogress and self.cylinder_rank == 0:
                print("")
                print("After PH Iteration", self._PHIter)
                print("Scaled PHBase Convergence Metric=", self.conv)
                print("Iteration time: %6.2f" % (time.time() - iteration_start_time))
                print("Elapsed time:   %6.2f" % (time.perf_counter() - self.start_time))
            if self.options["display_convergence_detail"]:
                self.report_var_values_at_rank0(header="Convergence detail:")
        else:
            self._settle()
            self.mpicomm.Barrier()
            if self.cylinder_rank == 0 and (dprogress or verbose):
                _global_toc("Reached user-specified limit=%d on number of PH iterations" % max_iterations)

    def post_loops(self, extensions=None):
        """phbase.py:982-1037."""
        verbose = self.options["verbose"]
        have_extensions = extensions is not None
        dprogress = self.options["display_progress"]
        dtiming = self.options["display_timing"]
        self._settle()
        self.mpicomm.Barrier()
        if self.scenario_denouement is not None:
            for sname, s in self.local_scenarios.items():
                target = self._models[sname] if self._models is not None else s
                self.scenario_denouement(self.cylinder_rank, sname, target)
        self.mpicomm.Barrier()
        if have_extensions:
            self.extobject.post_everything()
        if self.ph_converger is not None and hasattr(self.ph_converger, "post_everything"):
            self.convobject.post_everything()
        Eobj = self.Eobjective(verbose)
        self.mpicomm.Barrier()
        if dprogress and self.cylinder_rank == 0:
            print("")
            print("Current ***weighted*** E[objective] =", Eobj)
            print("")
        if dtiming and self.cylinder_rank == 0:
            print("")
            print("Cumulative execution time=%5.2f" % (time.perf_counter() - self.start_time))
            print("")
        return Eobj

    # ------------------------------------------------------------ accessors
    @property
    def _iter0_obj(self):
        """(S_local,) Iter0 subproblem optima, the reference's outer_bound after Iter0
        (spopt.py:201-206), in the model's sense."""
        return self._iter0_obj_dev.cpu().numpy() * (1.0 if self.is_minimizing else -1.0)

    def xbar_by_node(self):
        """{node_name: (xbar ndarray, xsqbar ndarray)} (host copy)."""
        xb = self._host("xbar")
        xs = self._host("xsqbar")
        out = {}
        for v, nd in enumerate(self._node_names):
            o, l = int(self._node_off[v]), int(self._node_nlen[v])
            out[nd] = (xb[o:o + l].copy(), xs[o:o + l].copy())
        return out

    def W_array(self):
        """(S_local, N) W values (host copy)."""
        return self._host("W").T.copy()
