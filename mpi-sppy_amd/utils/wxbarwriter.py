"""WXBarWriter extension (mpisppy/utils/wxbarwriter.py:26-101): after PH,
write W to ``options["W_fname"]`` (a directory when
``options["separate_W_files"]``) and x-bar to ``options["Xbar_fname"]``, in the
formats of utils/wxbarutils.py (appending to existing main files, as the
reference does)."""
import os

from ..extensions.extension import Extension
from . import wxbarutils


class WXBarWriter(Extension):
    def __init__(self, ph):
        super().__init__(ph)
        o = ph.options
        self.PHB = ph
        self.cylinder_rank = ph.cylinder_rank
        self.w_fname = o.get("W_fname")
        self.x_fname = o.get("Xbar_fname")
        self.sep_files = bool(o.get("separate_W_files", False))
        self.w_grad_fname = None
        root = self.cylinder_rank == 0
        if self.w_fname is None and self.x_fname is None and root:
            print("Warning: no output files provided to WXBarWriter. No values will be saved.")
        if self.w_fname and not self.sep_files and os.path.exists(self.w_fname) and root:
            print("Warning: specified W_fname ({fn}) already exists. Results will be appended to this file."
                  .format(fn=self.w_fname))
        elif self.w_fname and self.sep_files and not os.path.exists(self.w_fname) and root:
            print("Warning: path {p} does not exist. Creating...".format(p=self.w_fname))
            os.makedirs(self.w_fname, exist_ok=True)
        if self.x_fname and os.path.exists(self.x_fname) and root:
            print("Warning: specified Xbar_fname ({fn}) already exists. Results will be appended to this file."
                  .format(fn=self.x_fname))

    def post_everything(self):
        if self.w_fname:
            wxbarutils.write_W_to_file(self.PHB, self.w_fname, sep_files=self.sep_files)
        if self.x_fname:
            wxbarutils.write_xbar_to_file(self.PHB, self.x_fname)
