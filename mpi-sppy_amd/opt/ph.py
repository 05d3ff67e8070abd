"""PH — ``PH.ph_main`` (mirrors ``mpisppy/opt/ph.py:17-71``)."""
from ..phbase import PHBase


class PH(PHBase):
    """PH. See PHBase for list of args."""

    def ph_main(self, finalize=True):
        """Execute PH: PH_Prep -> subproblem_creation -> Iter0 -> iterk_loop -> post_loops.

        Returns (conv, Eobj, trivial_bound); Eobj is None when finalize=False.
        """
        verbose = self.options["verbose"]
        self.PH_Prep()
        self.subproblem_creation(verbose)
        # Iter0's E1 / feasibility checks and trivial bound may be evaluated right
        # after the device loop adopted its solve (PHBase._can_defer_iter0)
        self._defer_iter0_checks = True
        self.Iter0()
        if ("asynchronousPH" in self.options) and self.options["asynchronousPH"]:
            raise RuntimeError("asynchronousPH is deprecated; use APH")
        self.iterk_loop()
        if getattr(self, "_iter0_deferred", False):
            self._resolve_deferred_iter0()
        trivial_bound = self.trivial_bound
        Eobj = self.post_loops(self.extensions) if finalize else None
        return self.conv, Eobj, trivial_bound
