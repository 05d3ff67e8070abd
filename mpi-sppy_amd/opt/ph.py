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
        trivial_bound = self.Iter0()
        if ("asynchronousPH" in self.options) and self.options["asynchronousPH"]:
            raise RuntimeError("asynchronousPH is deprecated; use APH")
        self.iterk_loop()
        Eobj = self.post_loops(self.extensions) if finalize else None
        return self.conv, Eobj, trivial_bound
