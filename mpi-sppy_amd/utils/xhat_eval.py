"""Xhat_Eval — evaluate a candidate first-stage (nonant) solution.

Mirrors ``mpisppy.utils.xhat_eval.Xhat_Eval`` (``mpisppy/utils/xhat_eval.py:29-434``):
fix the nonants at a given ndn-keyed cache (lb = ub = value, applied to the
device batch by ``phx_set_bounds``), solve every local scenario in ONE batched
solve, and reduce ``E[obj]`` / ``infeas_prob`` / ``E[fct(obj)]``.

Differences from the reference, on purpose:
  * the reference's ``solve_one`` solves each scenario twice (its own
    ``super().solve_one`` and a second ``plugin.solve``, :82-107); here each
    evaluation is one batched solve;
  * ``evaluate_one`` solves the whole local batch (the batched solve costs the
    same for one scenario as for all) and returns the asked scenario's objective;
  * ``scenario_feasible`` is the batched solver's status (KKT-certified optimum)
    for both senses (the reference re-sets it to True only in its max branch,
    :119-124).
"""
import numpy as np
import torch

from ..spopt import SPOpt


class Xhat_Eval(SPOpt):
    """See SPOpt for the list of args."""

    def __init__(self, options, all_scenario_names, scenario_creator, scenario_denouement=None,
                 all_nodenames=None, mpicomm=None, scenario_creator_kwargs=None, variable_probability=None,
                 _native_lib=None, _device=None):
        super().__init__(options, all_scenario_names, scenario_creator,
                         scenario_denouement=scenario_denouement, all_nodenames=all_nodenames,
                         mpicomm=mpicomm, scenario_creator_kwargs=scenario_creator_kwargs,
                         variable_probability=variable_probability, _native_lib=_native_lib, _device=_device)
        self.verbose = self.options["verbose"]
        self.PH_extensions = None
        self._subproblems_solvers_created = False

    def _lazy_create_solvers(self):
        if self._subproblems_solvers_created:
            return
        self.subproblem_creation(self.verbose)
        self._create_solvers()
        self._subproblems_solvers_created = True

    # ------------------------------------------------------------ solves
    def solve_loop(self, solver_options=None, use_scenarios_not_subproblems=False, dtiming=False, gripe=False,
                   disable_pyomo_signal_handling=False, tee=False, verbose=False, compute_val_at_nonant=False):
        """One batched solve; with ``compute_val_at_nonant`` fills ``objs_dict``
        {scenario name: objective at the solution} (xhat_eval.py:140-215)."""
        self._lazy_create_solvers()
        super().solve_loop(solver_options, use_scenarios_not_subproblems, dtiming, gripe,
                           disable_pyomo_signal_handling, tee, verbose)
        if compute_val_at_nonant:
            self._fill_objs_dict()

    def _fill_objs_dict(self):
        self._objective_now()
        sgn = 1.0 if self.is_minimizing else -1.0
        vals = (self._obj_eval.cpu().numpy() + self._c0_int) * sgn
        self.objs_dict = {k: float(vals[s]) for s, k in enumerate(self.local_scenario_names)}

    def Eobjective(self, verbose=False, fct=None):
        """E[obj] or E[fct(obj)] over all scenarios (xhat_eval.py:218-263)."""
        self._lazy_create_solvers()
        if fct is None:
            return super().Eobjective(verbose=verbose)
        if not hasattr(self, "objs_dict"):
            raise RuntimeError("Values of the objective functions for each scenario"
                               " at xhat have to be computed before running Eobjective")
        local = []
        for s, k in enumerate(self.local_scenario_names):
            if k not in self.objs_dict:
                raise RuntimeError(f"No value has been calculated for the scenario {k}")
            local.append(float(self.batch.prob[s]) * np.asarray(fct(self.objs_dict[k]), dtype=np.float64))
        loc = np.atleast_1d(np.sum(np.array(local), axis=0))
        t = torch.as_tensor(loc, dtype=torch.float64, device=self.device)
        self.mpicomm.allreduce_(t)
        g = t.cpu().numpy()
        return float(g[0]) if len(g) == 1 else g

    def evaluate_one(self, nonant_cache, scenario_name, s):
        """Objective of one scenario at the fixed xhat (xhat_eval.py:266-295)."""
        self._lazy_create_solvers()
        self._fix_nonants(nonant_cache)
        if not hasattr(self, "objs_dict"):
            self.objs_dict = {}
        solver_options = self.options["solver_options"] if "solver_options" in self.options else None
        self.solve_loop(solver_options=solver_options, gripe=True, verbose=self.verbose,
                        compute_val_at_nonant=True)
        return self.objs_dict[scenario_name]

    def evaluate(self, nonant_cache, fct=None):
        """Fix xhat, solve, return E[obj] (or E[fct(obj)]) (xhat_eval.py:297-327)."""
        self._lazy_create_solvers()
        self._fix_nonants(nonant_cache)
        solver_options = self.options["solver_options"] if "solver_options" in self.options else None
        self.solve_loop(solver_options=solver_options, use_scenarios_not_subproblems=True, gripe=True,
                        tee=False, verbose=self.verbose, compute_val_at_nonant=True)
        return self.Eobjective(self.verbose, fct=fct)

    def fix_nonants_upto_stage(self, t, cache):
        """Fix the nonants of stages 1..t at ``cache[ndn]`` (xhat_eval.py:331-366)."""
        self._lazy_create_solvers()
        vals, mask = self._cache_by_slot(cache, stage_max=t)
        self._fix_where(vals, mask)

    def _fix_nonants_at_value(self):
        """Fix every nonant at its current value (xhat_eval.py:371-404)."""
        x = self._nonant_x()
        self._fix_where(x, np.ones(x.shape, dtype=bool))

    def calculate_incumbent(self, fix_nonants=True, verbose=False):
        """E[obj] with the nonants fixed at their current values, or None if
        some scenario is infeasible (xhat_eval.py:406-430)."""
        self._lazy_create_solvers()
        if fix_nonants:
            self._fix_nonants_at_value()
        self.solve_loop(solver_options=self.current_solver_options, verbose=verbose)
        infeasP = self.infeas_prob()
        if infeasP != 0.:
            return None
        if verbose and self.cylinder_rank == 0:
            print("  Feasible xhat found")
        return self.Eobjective(verbose=verbose)
