"""Node-local one-sided windows for the hub <-> spoke wire format.

Replaces ``SPCommunicator._make_window`` (spcommunicator.py:93-120: an
``MPI.Win.Allocate`` of ``length + 1`` doubles, the last one the write id) and
the ``Lock / Put / Unlock`` and ``Lock / Get / Unlock`` epochs of
hub.py:370-450 and spoke.py:60-118.

One process per GPU on ONE node (the MI355X deployment), so a window is a POSIX
shared-memory segment owned by one strata rank: the owner is the only writer
(the reference's convention: a process Puts into its own buffer, the peer Gets
from it).  An epoch is a sequence lock instead of an MPI lock: the writer makes
the sequence word odd, writes the payload, makes it even again; a reader copies
the payload and retries if the word was odd or changed meanwhile.  A writer
never waits for a slow reader (the hub keeps iterating while a spoke reads),
and a reader always sees one complete write — the guarantee the MPI lock gave.

Segment layout (bytes): [seq: int64 | payload: (length + 1) float64].

Memory ordering: the sequence word and the payload are plain numpy stores and
loads, with no explicit fences.  The lock is correct on the deployment host
(x86-64, EPYC: total store order — stores become visible in program order and
loads are not reordered with older loads), and CPython executes each store as
a separate C call the compiler cannot move across.  ``_check_host`` refuses to
build a window on any other architecture rather than run an unfenced seqlock
there.

Crash cleanup: every segment this process created is registered with
``atexit`` and unlinked there if ``free`` never ran, so a spoke that dies with
an exception does not leave its segments in /dev/shm (a SIGKILL still can; the
names are per tag, and a new window with the same name truncates the old
file).
"""
import atexit
import mmap
import os
import platform
import time

import numpy as np

_SHM_DIR = "/dev/shm"
_OWNED = set()          # paths of segments this process created and has not unlinked


def _check_host():
    m = platform.machine().lower()
    if m not in ("x86_64", "amd64"):
        raise RuntimeError("SPWindow's sequence lock relies on x86-64 store ordering; host is %s" % m)


@atexit.register
def _unlink_owned():
    for path in list(_OWNED):
        try:
            os.unlink(path)
        except FileNotFoundError:
            pass
        _OWNED.discard(path)


class _Segment:
    """A named POSIX shared-memory file mapped into this process (no Python
    resource tracker: only the owner unlinks, in ``SPWindow.free``)."""

    def __init__(self, name, size=None):
        self.path = os.path.join(_SHM_DIR, name)
        if size is not None:
            _check_host()
            fd = os.open(self.path, os.O_RDWR | os.O_CREAT | os.O_TRUNC, 0o600)
            _OWNED.add(self.path)
            os.ftruncate(fd, size)
        else:
            fd = os.open(self.path, os.O_RDWR)
            size = os.fstat(fd).st_size
        try:
            self.buf = mmap.mmap(fd, size)
        finally:
            os.close(fd)

    def close(self):
        self.buf.close()

    def unlink(self):
        _OWNED.discard(self.path)
        os.unlink(self.path)


class SPWindow:
    """One window: a segment per strata rank (zero-length for ranks that do not
    own a buffer in it).  ``put`` writes this rank's own buffer, ``get(owner)``
    reads another rank's."""

    def __init__(self, tag, index, my_rank, lengths):
        """lengths[r]: payload length (WITHOUT the write-id slot) that strata
        rank r owns in this window.  Collective in the sense that every rank
        creates its own segment first; ``attach`` opens the peers' after a
        barrier."""
        self.tag = tag
        self.index = index
        self.rank = my_rank
        self.lengths = list(lengths)
        self._own = self._create(my_rank, self.lengths[my_rank])
        self._peers = {}
        self.buffer = self._payload(self._own, self.lengths[my_rank])
        self.buffer[-1] = 0.0             # write id starts at zero (spcommunicator.py:119)

    def _name(self, r):
        return "phxw_%s_%d_%d" % (self.tag, self.index, r)

    @staticmethod
    def _nbytes(length):
        return 8 + 8 * (length + 1)

    def _create(self, r, length):
        shm = _Segment(self._name(r), size=self._nbytes(length))
        np.ndarray((1,), dtype=np.int64, buffer=shm.buf)[0] = 0
        return shm

    @staticmethod
    def _seq(shm):
        return np.ndarray((1,), dtype=np.int64, buffer=shm.buf)

    @staticmethod
    def _payload(shm, length):
        return np.ndarray((length + 1,), dtype=np.float64, buffer=shm.buf, offset=8)

    def attach(self, r):
        """Open strata rank r's segment (after every owner created its own)."""
        if r == self.rank:
            return self._own
        if r not in self._peers:
            self._peers[r] = _Segment(self._name(r))
        return self._peers[r]

    def put(self, values):
        """Write ``values`` (length + 1, write id included) into this rank's
        own buffer: one seqlock epoch."""
        seq = self._seq(self._own)
        s = int(seq[0])
        seq[0] = s + 1                    # odd: write in progress
        self.buffer[:] = values
        seq[0] = s + 2

    def get(self, r, out, timeout=60.0):
        """Copy strata rank r's buffer into ``out`` (one consistent epoch)."""
        shm = self.attach(r)
        seq = self._seq(shm)
        src = self._payload(shm, self.lengths[r])
        t0 = time.monotonic()
        while True:
            s1 = int(seq[0])
            if s1 & 1 == 0:
                out[:] = src
                if int(seq[0]) == s1:
                    return out
            if time.monotonic() - t0 > timeout:
                raise RuntimeError("SPWindow %s: writer of rank %d never finished an epoch" % (self._name(r), r))
            os.sched_yield()

    def free(self):
        for shm in self._peers.values():
            shm.close()
        self._peers = {}
        self.buffer = None
        self._own.close()
        try:
            self._own.unlink()
        except FileNotFoundError:
            pass
