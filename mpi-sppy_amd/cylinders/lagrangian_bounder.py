"""Lagrangian outer-bound spoke (cylinders/lagrangian_bounder.py:5-95).

The spoke's opt object is a PHBase (cfg_vanilla.lagrangian_spoke): PH_Prep
without the prox term, W enabled, one batched solve of all local scenarios per
new W vector the hub sends (the same device solve as the hub's, prox off), and
``Ebound`` with the write id as an extra sum term so the bound is used only
when every cylinder rank solved with W of the same hub iteration.
"""
from .spoke import OuterBoundWSpoke


class LagrangianOuterBound(OuterBoundWSpoke):
    converger_spoke_char = "L"

    def lagrangian_prep(self):
        verbose = self.opt.options["verbose"]
        self.opt.PH_Prep(attach_prox=False)
        self.opt._reenable_W()
        self.opt.subproblem_creation(verbose)
        self.opt._create_solvers()

    def lagrangian(self):
        verbose = self.opt.options["verbose"]
        if "ipopt" in self.opt.options["solver_name"]:
            print("\n WARNING: An ipopt solver will not give outer bounds\n")
        teeme = bool(self.opt.options.get("tee-rank0-solves", False))
        self.opt.solve_loop(solver_options=self.opt.current_solver_options, dtiming=False, gripe=True,
                            tee=teeme, verbose=verbose)
        # the bound, checking that the weights came from the same PH iteration
        serial_number = self.get_serial_number()
        bound, extra_sums = self.opt.Ebound(verbose, extra_sum_terms=[serial_number])
        serial_number_sum = int(round(extra_sums[0]))
        total = int(self.cylinder_comm.Get_size()) * serial_number
        if total == serial_number_sum:
            return bound
        elif self.cylinder_rank == 0:
            raise RuntimeError("Lagrangian spokes unexpectly out of snyc")
        return None

    def _set_weights_and_solve(self):
        self.opt.W_from_flat_list(self.localWs)
        return self.lagrangian()

    def main(self):
        self.lagrangian_prep()
        self.dk_iter = 1
        self.trivial_bound = self.lagrangian()
        self.opt.current_solver_options = self.opt.iterk_solver_options
        self.bound = self.trivial_bound
        while not self.got_kill_signal():
            if self.new_Ws:
                bound = self._set_weights_and_solve()
                if bound is not None:
                    self.bound = bound
                self.dk_iter += 1

    def finalize(self):
        """One last pass with the last W vector read (lagrangian_bounder.py:84-95)."""
        self.final_bound = self._set_weights_and_solve()
        self.bound = self.final_bound
        if self.opt.extensions is not None and hasattr(self.opt.extobject, "post_everything"):
            self.opt.extobject.post_everything()
        return self.final_bound
