"""Lagrangian outer-bound spoke (the role of mpisppy/cylinders/lagrangian_bounder.py:5-95).

Its opt object is a PHBase (cfg_vanilla.lagrangian_spoke).  Each W vector the
hub publishes defines the Lagrangian relaxation min_x sum_s p_s (f_s(x_s) +
W_s x_s) -- the PH objective without the prox term -- whose value is a valid
outer bound.  The spoke evaluates it with one batched device solve of all
local scenarios and reports sum_s p_s f*_s through Ebound.  The hub tags every
W vector with its write id; the bound counts only if every rank of this
cylinder solved with the vector of the same tag (the tag rides along as an
extra term of the Ebound all-reduce: its sum must be cylinder size x tag).
"""
from .spoke import OuterBoundWSpoke


class LagrangianOuterBound(OuterBoundWSpoke):
    converger_spoke_char = "L"

    def lagrangian_prep(self):
        """PH objective terms with W on and prox off, the solver objects."""
        opt = self.opt
        opt.PH_Prep(attach_prox=False)
        opt._reenable_W()
        opt.subproblem_creation(opt.options["verbose"])
        opt._create_solvers()

    def lagrangian(self):
        """Solve with the current W; the bound, or None when the cylinder's
        ranks did not all hold the same hub vector."""
        opt = self.opt
        if "ipopt" in opt.options["solver_name"]:
            print("\n WARNING: An ipopt solver will not give outer bounds\n")
        opt.solve_loop(solver_options=opt.current_solver_options, dtiming=False, gripe=True,
                       tee=bool(opt.options.get("tee-rank0-solves", False)), verbose=opt.options["verbose"])
        tag = self.get_serial_number()
        bound, (tag_sum,) = opt.Ebound(opt.options["verbose"], extra_sum_terms=[tag])
        if int(round(tag_sum)) == self.cylinder_comm.Get_size() * tag:
            return bound
        if self.cylinder_rank == 0:
            raise RuntimeError("Lagrangian spoke: the cylinder's ranks solved with W vectors of different "
                               "hub iterations")
        return None

    def _bound_for(self, flat_W):
        self.opt.W_from_flat_list(flat_W)
        return self.lagrangian()

    def main(self):
        self.lagrangian_prep()
        self.dk_iter = 1
        self.trivial_bound = self.lagrangian()          # W = 0: the trivial bound
        self.opt.current_solver_options = self.opt.iterk_solver_options
        self.bound = self.trivial_bound
        while not self.got_kill_signal():
            if not self.new_Ws:
                continue
            b = self._bound_for(self.localWs)
            if b is not None:
                self.bound = b
            self.dk_iter += 1

    def finalize(self):
        """One more bound from the last W vector read."""
        self.final_bound = self._bound_for(self.localWs)
        self.bound = self.final_bound
        ext = self.opt.extensions
        if ext is not None and hasattr(self.opt.extobject, "post_everything"):
            self.opt.extobject.post_everything()
        return self.final_bound
