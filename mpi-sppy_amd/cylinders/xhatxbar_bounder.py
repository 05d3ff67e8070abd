"""x-bar inner-bound spoke (cylinders/xhatxbar_bounder.py:31-114).

Its opt object is an Xhat_Eval; every new nonant vector from the hub becomes
the current nonants, x-bar of those is fixed and evaluated by one batched
solve (extensions/xhatxbar.py), and an improving objective is sent to the hub
as an inner bound.
"""
from ..extensions.xhatxbar import XhatXbar
from ..utils.xhat_eval import Xhat_Eval
from .spoke import InnerBoundNonantSpoke


class XhatXbarInnerBound(InnerBoundNonantSpoke):
    converger_spoke_char = "B"

    def ib_prep(self):
        if "bundles_per_rank" in self.opt.options and self.opt.options["bundles_per_rank"] != 0:
            raise RuntimeError("xhat spokes cannot have bundles (yet)")
        if not isinstance(self.opt, Xhat_Eval):
            raise RuntimeError("XhatXbarInnerBound must be used with Xhat_Eval.")
        xhatter = XhatXbar(self.opt)
        xhatter.pre_iter0()
        self.opt._save_original_nonants()
        self.opt._lazy_create_solvers()
        self.opt._update_E1()
        if abs(1 - self.opt.E1) > self.opt.E1_tolerance:
            if self.opt.cylinder_rank == 0:
                print("ERROR")
                print("Total probability of scenarios was ", self.opt.E1)
                print("E1_tolerance = ", self.opt.E1_tolerance)
            quit()
        xhatter.post_iter0()
        self.opt._save_nonants()
        return xhatter

    def main(self):
        xhatter = self.ib_prep()
        self.ib_iter = 1
        while not self.got_kill_signal():
            if self.new_nonants:
                self.opt._put_nonant_cache(self.localnonants)
                self.opt._restore_nonants()
                innerbound = xhatter.xhat_tryit(restore_nonants=False)
                self.update_if_improving(innerbound)
            self.ib_iter += 1
