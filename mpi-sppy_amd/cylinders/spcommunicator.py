"""SPCommunicator: the base of hubs and spokes (spcommunicator.py:21-120).

Same constructor and methods; communicators are ``mpisppy_amd.comm.Comm``
objects (torch.distributed groups: RCCL on GPUs, gloo on CPU) and windows are
node-local shared-memory segments (``spwindow.SPWindow``) instead of MPI RMA
windows.  The star topology is the reference's: spokes talk to the hub only.
"""
import time
import uuid

import numpy as np

from .spwindow import SPWindow


def window_lengths(hub_lengths, spoke_lengths):
    """Per-window owner lengths: window i (spoke i + 1) holds the hub's buffer
    for that spoke (hub_lengths[i] payload values, owned by strata rank 0) and
    the spoke's own buffer (spoke_lengths[i], owned by strata rank i + 1);
    the other strata ranks own nothing in it."""
    n = len(hub_lengths)
    out = []
    for i in range(n):
        ln = [0] * (n + 1)
        ln[0] = int(hub_lengths[i])
        ln[i + 1] = int(spoke_lengths[i])
        out.append(ln)
    return out


class SPCommunicator:
    def __init__(self, spbase_object, fullcomm, strata_comm, cylinder_comm, options=None):
        self._windows_constructed = False
        self.fullcomm = fullcomm
        self.strata_comm = strata_comm
        self.cylinder_comm = cylinder_comm
        self.global_rank = fullcomm.Get_rank()
        self.strata_rank = strata_comm.Get_rank()
        self.cylinder_rank = cylinder_comm.Get_rank()
        self.n_spokes = strata_comm.Get_size() - 1
        self.opt = spbase_object
        self.inst_time = time.time()
        self.options = dict() if options is None else options
        # attach the SPCommunicator to the SPBase object (a weakref there)
        self.opt.spcomm = self

    def main(self):
        raise NotImplementedError

    def sync(self):
        pass

    def is_converged(self):
        return False

    def finalize(self):
        pass

    def hub_finalize(self):
        pass

    def allreduce_or(self, val):
        g = self.cylinder_comm.allreduce_np(np.array([1 if val else 0], dtype=np.int64), op="max")
        return bool(g[0] > 0)

    def _window_tag(self):
        """One tag per strata group, agreed through the strata communicator
        (segment names must match between the hub and its spokes)."""
        tag = uuid.uuid4().hex[:12] if self.strata_rank == 0 else None
        return "%s_%d" % (self.strata_comm.bcast(tag, root=0), self.cylinder_rank)

    def _make_windows_from_lengths(self, lengths_per_window):
        """lengths_per_window[i][r]: payload length strata rank r owns in
        window i (one window per spoke).  Every strata rank creates its own
        segments, then (barrier) opens the peers'."""
        tag = self._window_tag()
        self.windows = [SPWindow(tag, i, self.strata_rank, lengths_per_window[i]) for i in range(self.n_spokes)]
        self.buffers = [w.buffer for w in self.windows]
        self.strata_comm.Barrier()
        for i, w in enumerate(self.windows):
            for r, ln in enumerate(lengths_per_window[i]):
                if r != self.strata_rank and ln > 0:
                    w.attach(r)
        self.strata_comm.Barrier()
        self._windows_constructed = True

    def free_windows(self):
        if self._windows_constructed:
            self.strata_comm.Barrier()    # nobody reads a segment its owner unlinks
            del self.buffers
            for w in self.windows:
                w.free()
        self._windows_constructed = False
