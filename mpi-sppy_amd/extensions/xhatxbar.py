"""XhatXbar: try x-bar as the incumbent (extensions/xhatxbar.py:12-120).

The nonants of every local scenario are fixed at the x-bar of their tree node
(computed from the opt object's current nonant values: phbase._Compute_Xbar,
phbase.py:27-107, on the device), all scenarios are solved in one batched
solve, and the objective is returned when every scenario is feasible
(infeas_prob == 0), else None.  The engine's models are continuous (LP/QP
relaxations), so the reference's rounding of integer nonants never applies.
"""
import numpy as np
import torch


class XhatXbar:
    def __init__(self, spo):
        self.opt = spo
        self.cylinder_rank = spo.cylinder_rank
        self.options = spo.options["xhat_xbar_options"]
        self.solver_options = self.options["xhat_solver_options"]
        self.keep_solution = not ("keep_solution" in self.options and not self.options["keep_solution"])

    def _xbar_by_slot(self):
        """(S_local, N) x-bar of each scenario's node per nonant slot, from the
        current nonant values (one device reduction + all-reduce)."""
        opt = self.opt
        opt._settle()
        lib = opt._native
        lib.check(opt._ctx, lib.xbar(opt._ctx, opt._tree, opt._x.data_ptr(), opt._pc.data_ptr(),
                                     opt._partial.data_ptr(), opt._node_buf.data_ptr(), opt._stream()), "xbar")
        opt.mpicomm.allreduce_(opt._node_buf)
        xb = opt._xbar_node[opt._xbar_idx_t.long()]          # [N*S], slot-major
        return xb.view(-1, opt._S).t().cpu().numpy()

    def _fix_nonants_xhat(self):
        vals = self._xbar_by_slot()
        self.opt._fix_where(vals, np.ones(vals.shape, dtype=bool))

    def xhat_tryit(self, verbose=False, restore_nonants=True):
        """x-bar as xhat: E[obj] or None if infeasible (xhatxbar.py:57-112)."""
        def _vb(msg):
            if verbose and self.cylinder_rank == 0:
                print("  xhat_xbar: " + msg)
        _vb("Enter XhatXbar.xhat_tryit")
        self._fix_nonants_xhat()
        self.opt.solve_loop(solver_options=self.solver_options, verbose=verbose, tee=False)
        infeasP = self.opt.infeas_prob()
        if infeasP != 0.:
            self.opt._restore_nonants()
            _vb("Infeasible")
            return None
        obj = self.opt.Eobjective(verbose=verbose)
        if restore_nonants:
            self.opt._restore_nonants()
        _vb("Feasible, returning " + str(obj))
        return obj

    def pre_iter0(self):
        pass

    def post_iter0(self):
        self.comms = self.opt.comms

    def miditer(self):
        pass

    def enditer(self):
        pass

    def post_everything(self):
        pass
