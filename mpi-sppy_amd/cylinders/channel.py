"""One direction of a hub <-> spoke window, as an object.

The reference spreads the wire protocol over ``Hub.hub_to_spoke`` /
``hub_from_spoke`` (hub.py:370-436) and ``Spoke.spoke_to_hub`` /
``spoke_from_hub`` (spoke.py:60-118), each with its own write-id counter and
its own agreement test.  Here both ends use the same two classes:

* ``Outbox`` -- the owner's side of one buffer (owner = the rank that writes
  it, as in the reference: a process only ever writes its own buffer).
  ``publish(buf)`` stamps ``buf[-1]`` with the next write id and puts it;
  ``kill(length)`` puts zeros with write id -1 (the reference's termination
  signal, hub.py:438-450).
* ``Inbox`` -- the reader's side.  ``poll(buf)`` copies the buffer out of the
  window and reports whether it is NEW: every rank of the reading cylinder
  must have read the same write id (one max-all-reduce of ``(id, -id)``:
  max == min), and that id must be newer than the last one accepted or
  negative (the kill signal is always news).

Wire format (unchanged, the reference's): a flat fp64 buffer whose last slot
is the write id.  Hub -> spoke payloads end with ``[outer, inner, write_id]``.
"""
import numpy as np


class _Box:
    def __init__(self, window, owner, length, cylinder_comm):
        self.window = window          # spwindow.SPWindow
        self.owner = owner            # strata rank that writes the buffer
        self.length = int(length)     # payload length, write id excluded
        self.comm = cylinder_comm

    def _check(self, buf, who):
        if len(buf) != self.length + 1:
            raise RuntimeError("%s: buffer of length %d for a window of %d payload values (+ write id)"
                               % (who, len(buf), self.length))


class Outbox(_Box):
    """The owner's side of a buffer."""

    def __init__(self, window, owner, length, cylinder_comm):
        super().__init__(window, owner, length, cylinder_comm)
        self.write_id = 0

    def publish(self, buf):
        self._check(buf, "Outbox.publish")
        # every rank of the writing cylinder stamps the same id at about the
        # same time (the readers' agreement test compares them)
        self.comm.Barrier()
        self.write_id += 1
        buf[-1] = self.write_id
        self.window.put(buf)

    def kill(self):
        buf = np.zeros(self.length + 1)
        buf[-1] = -1
        self.window.put(buf)


class Inbox(_Box):
    """The reader's side of a buffer."""

    def __init__(self, window, owner, length, cylinder_comm):
        super().__init__(window, owner, length, cylinder_comm)
        self.read_id = 0

    def poll(self, buf):
        self._check(buf, "Inbox.poll")
        self.comm.Barrier()
        self.window.get(self.owner, buf)
        wid = int(buf[-1])
        hi = self.comm.allreduce_np(np.array([wid, -wid], dtype=np.int64), op="max")
        if int(hi[0]) != -int(hi[1]):
            return False              # the ranks caught different writes: wait for the next
        if wid < 0 or wid > self.read_id:
            self.read_id = wid
            return True
        return False

    @property
    def killed(self):
        return self.read_id == -1
