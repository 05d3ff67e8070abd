"""Spokes: the cylinders that read what the hub publishes and send bounds back
(the reference's class hierarchy of mpisppy/cylinders/spoke.py:18-376 -- same
class names, roles and attributes -- built here on two channel objects).

A spoke owns one window (the one of its strata rank):

* ``to_hub``   an ``Outbox`` it owns: ``[bound | write_id]`` (one value);
* ``from_hub`` an ``Inbox`` the hub owns: ``[payload | outer, inner, write_id]``,
  where the payload is W or the nonants of this rank's scenarios (scenario-major,
  the reference's flat layout) or empty for bound-only spokes.

The class decides the payload by its roles (``converger_spoke_types``), the
hub reads the same roles to decide what to publish (hub.py).  Every poll of
the hub's buffer goes through ``got_kill_signal()``; ``new_Ws`` /
``new_nonants`` report whether that poll brought a new vector.
"""
import enum
import math
import os
import time

import numpy as np

from .channel import Inbox, Outbox
from .spcommunicator import SPCommunicator, window_lengths


class ConvergerSpokeType(enum.Enum):
    OUTER_BOUND = 1
    INNER_BOUND = 2
    W_GETTER = 3
    NONANT_GETTER = 4


class Spoke(SPCommunicator):
    """Base spoke: the two channels and the length handshake."""

    # payload length the spoke wants from the hub: "none" (bounds only) or
    # "per_nonant" (one value per local nonant: W or nonants)
    hub_payload = "none"

    def __init__(self, spbase_object, fullcomm, strata_comm, cylinder_comm, options=None):
        super().__init__(spbase_object, fullcomm, strata_comm, cylinder_comm, options)
        self.to_hub = None
        self.from_hub = None
        self._hub_buf = None          # last buffer read from the hub (payload | outer, inner, id)
        self._fresh = False           # the last poll brought a new buffer

    # ---- window setup: announce (own length, wanted length); the hub answers
    #      with its own announcement (None) in the same all-gather
    def _payload_length(self):
        if self.hub_payload == "none":
            return 0
        scen = getattr(self.opt, "local_scenarios", None)
        if scen is None:
            raise RuntimeError("this spoke needs an opt object with local_scenarios")
        if len(scen) == 0:
            raise RuntimeError("Rank has zero local_scenarios")
        return len(scen) * self.opt.batch.nonant.N

    def make_windows(self):
        mine = 1                                          # the bound
        wanted = self._payload_length() + 2               # + outer, inner
        ann = self.strata_comm.allgather_object((mine, wanted))
        spokes = ann[1:]
        self._make_windows_from_lengths(window_lengths([w for _, w in spokes], [m for m, _ in spokes]))
        win = self.windows[self.strata_rank - 1]
        self.to_hub = Outbox(win, self.strata_rank, mine, self.cylinder_comm)
        self.from_hub = Inbox(win, 0, wanted, self.cylinder_comm)
        self._hub_buf = np.zeros(wanted + 1)
        self._bound_buf = np.zeros(mine + 1)

    # ---- the reference's names for the two directions
    @property
    def local_write_id(self):
        return self.to_hub.write_id if self.to_hub else 0

    @property
    def remote_write_id(self):
        return self.from_hub.read_id if self.from_hub else 0

    @property
    def local_length(self):
        return self.to_hub.length if self.to_hub else 0

    @property
    def remote_length(self):
        return self.from_hub.length if self.from_hub else 0

    def spoke_to_hub(self, values):
        self.to_hub.publish(values)

    def spoke_from_hub(self, values):
        return self.from_hub.poll(values)

    def got_kill_signal(self):
        """Poll the hub's buffer once; True when it carries the kill signal."""
        self._fresh = self.from_hub.poll(self._hub_buf)
        return self.from_hub.killed

    def get_serial_number(self):
        """The write id of the last hub buffer accepted (its PH iteration tag)."""
        return self.remote_write_id

    def main(self):
        raise NotImplementedError


class _BoundSpoke(Spoke):
    """A spoke that sends one bound (optionally traced to a CSV file)."""

    def __init__(self, spbase_object, fullcomm, strata_comm, cylinder_comm, options=None):
        super().__init__(spbase_object, fullcomm, strata_comm, cylinder_comm, options)
        self.trace_filen = None
        opts = getattr(spbase_object, "options", None) or {}
        prefix = opts.get("trace_prefix")
        if prefix is not None and self.cylinder_rank == 0:
            self.trace_filen = prefix + type(self).__name__ + ".csv"
            if os.path.exists(self.trace_filen):
                raise RuntimeError("spoke trace file %s exists already" % self.trace_filen)
            with open(self.trace_filen, "w") as f:
                f.write("time,bound\n")
            self.start_time = spbase_object.start_time

    @property
    def bound(self):
        return self._bound_buf[0]

    @bound.setter
    def bound(self, value):
        if self.trace_filen is not None:
            with open(self.trace_filen, "a") as f:
                f.write("%r,%r\n" % (time.perf_counter() - self.start_time, value))
        self._bound_buf[0] = value
        self.to_hub.publish(self._bound_buf)

    @property
    def hub_outer_bound(self):
        return self._hub_buf[-3]

    @property
    def hub_inner_bound(self):
        return self._hub_buf[-2]

    @property
    def _payload(self):
        return self._hub_buf[:-3]


class InnerBoundSpoke(_BoundSpoke):
    converger_spoke_types = (ConvergerSpokeType.INNER_BOUND,)
    converger_spoke_char = "I"


class OuterBoundSpoke(_BoundSpoke):
    converger_spoke_types = (ConvergerSpokeType.OUTER_BOUND,)
    converger_spoke_char = "O"


class OuterBoundWSpoke(_BoundSpoke):
    """Receives W of every local scenario (scenario-major) with the bounds."""
    converger_spoke_types = (ConvergerSpokeType.OUTER_BOUND, ConvergerSpokeType.W_GETTER)
    converger_spoke_char = "O"
    hub_payload = "per_nonant"

    @property
    def localWs(self):
        return self._payload

    @property
    def new_Ws(self):
        return self._fresh


class _NonantSpoke(_BoundSpoke):
    hub_payload = "per_nonant"

    @property
    def localnonants(self):
        return self._payload

    @property
    def new_nonants(self):
        return self._fresh


class InnerBoundNonantSpoke(_NonantSpoke):
    """Receives the hub's nonants, sends incumbents (inner bounds); keeps the
    device solution of the best incumbent so finalize() can restore it."""
    converger_spoke_types = (ConvergerSpokeType.INNER_BOUND, ConvergerSpokeType.NONANT_GETTER)
    converger_spoke_char = "I"

    def __init__(self, spbase_object, fullcomm, strata_comm, cylinder_comm, options=None):
        super().__init__(spbase_object, fullcomm, strata_comm, cylinder_comm, options)
        self.is_minimizing = self.opt.is_minimizing
        self.best_inner_bound = math.inf if self.is_minimizing else -math.inf
        self.solver_options = None
        self.best_solution_cache = None

    def _better(self, value):
        return value < self.best_inner_bound if self.is_minimizing else value > self.best_inner_bound

    def update_if_improving(self, candidate_inner_bound):
        """Send the candidate if it improves on the best so far (and cache the
        solution that produced it); returns whether it did."""
        if candidate_inner_bound is None or not self._better(candidate_inner_bound):
            return False
        self.best_inner_bound = candidate_inner_bound
        self.bound = candidate_inner_bound
        self.opt._settle()
        self.best_solution_cache = self.opt._x.clone()
        return True

    def finalize(self):
        if self.best_solution_cache is None:
            return None
        self.opt._settle()
        self.opt._x.copy_(self.best_solution_cache)
        self.opt._bump()
        self.opt.first_stage_solution_available = True
        self.opt.tree_solution_available = True
        self.final_bound = self.bound
        return self.final_bound


class OuterBoundNonantSpoke(_NonantSpoke):
    converger_spoke_types = (ConvergerSpokeType.OUTER_BOUND, ConvergerSpokeType.NONANT_GETTER)
    converger_spoke_char = "A"
