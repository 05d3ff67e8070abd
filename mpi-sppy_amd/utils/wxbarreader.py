"""WXBarReader extension (mpisppy/utils/wxbarreader.py:25-97): at PH iteration
1, after Compute_Xbar / Update_W and before the solve (``miditer``), replace W
with ``options["init_W_fname"]`` (a directory of ``<sname>_weights.csv`` when
``options["init_separate_W_files"]``) and x-bar with
``options["init_Xbar_fname"]``, re-enabling the W / prox terms.  A named file
that does not exist ends the run, as the reference's ``quit()`` does."""
import os
import sys

from ..extensions.extension import Extension
from . import wxbarutils


class WXBarReader(Extension):
    def __init__(self, ph):
        super().__init__(ph)
        o = ph.options
        self.PHB = ph
        self.cylinder_rank = ph.cylinder_rank
        self.sep_files = bool(o.get("init_separate_W_files", False))
        self.w_fname = o.get("init_W_fname")
        self.x_fname = o.get("init_Xbar_fname")
        root = self.cylinder_rank == 0
        for fn, what in ((self.w_fname, "path" if self.sep_files else "file"), (self.x_fname, "file")):
            if fn is not None and not os.path.exists(fn):
                if root:
                    print("Cannot find %s" % what, fn)
                sys.exit()
        if self.w_fname is None and self.x_fname is None and root:
            print("Warning: no input files provided to WXBarReader. "
                  "W and Xbar will be initialized to their default values.")

    def miditer(self):
        if self.PHB._PHIter == 1:
            if self.w_fname:
                wxbarutils.set_W_from_file(self.w_fname, self.PHB, self.cylinder_rank, sep_files=self.sep_files)
                self.PHB._reenable_W()
            if self.x_fname:
                wxbarutils.set_xbar_from_file(self.x_fname, self.PHB)
                self.PHB._reenable_prox()
