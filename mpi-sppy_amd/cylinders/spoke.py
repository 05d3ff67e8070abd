"""Spoke side of the hub-and-spoke system (cylinders/spoke.py:18-376).

Same class hierarchy and wire format as the reference: a spoke owns one buffer
``[bound | write_id]`` (spoke -> hub) and reads the hub's ``[payload | outer,
inner, write_id]`` (hub -> spoke); ``spoke_from_hub`` accepts a read only when
every cylinder rank saw the same write id (max == min over the cylinder,
spoke.py:84-118), and ``write_id == -1`` is the kill signal.
"""
import enum
import math
import os
import time

import numpy as np

from .spcommunicator import SPCommunicator


class ConvergerSpokeType(enum.Enum):
    OUTER_BOUND = 1
    INNER_BOUND = 2
    W_GETTER = 3
    NONANT_GETTER = 4


class Spoke(SPCommunicator):
    def __init__(self, spbase_object, fullcomm, strata_comm, cylinder_comm, options=None):
        super().__init__(spbase_object, fullcomm, strata_comm, cylinder_comm, options)
        self.local_write_id = 0
        self.remote_write_id = 0
        self.local_length = 0      # does NOT include the + 1
        self.remote_length = 0     # length on the hub; does NOT include + 1
        self.last_call_to_got_kill_signal = time.time()

    def _make_windows(self, local_length, remote_length):
        """spoke.py:34-58: tell the hub the two lengths, then build the windows."""
        from .hub import _window_lengths
        pairs = self.strata_comm.allgather_object((int(local_length), int(remote_length)))
        self.local_length = local_length
        self.remote_length = remote_length
        spoke_lengths = [pairs[i + 1][0] for i in range(self.n_spokes)]
        hub_lengths = [pairs[i + 1][1] for i in range(self.n_spokes)]
        self._make_windows_from_lengths(_window_lengths(self.n_spokes, hub_lengths, spoke_lengths))

    def spoke_to_hub(self, values):
        """spoke.py:60-82."""
        expected = self.local_length + 1
        if len(values) != expected:
            raise RuntimeError(f"Attempting to put array of length {len(values)} "
                               f"into local buffer of length {expected}")
        self.cylinder_comm.Barrier()
        self.local_write_id += 1
        values[-1] = self.local_write_id
        self.windows[self.strata_rank - 1].put(values)

    def spoke_from_hub(self, values):
        """spoke.py:84-118."""
        expected = self.remote_length + 1
        if len(values) != expected:
            raise RuntimeError(f"Spoke trying to get buffer of length {expected} "
                               f"from hub, but provided buffer has length {len(values)}.")
        self.cylinder_comm.Barrier()
        self.windows[self.strata_rank - 1].get(0, values)
        new_id = int(values[-1])
        mm = self.cylinder_comm.allreduce_np(np.array([new_id, -new_id], dtype=np.int64), op="max")
        max_id, min_id = int(mm[0]), -int(mm[1])
        # only proceed if all the ranks agree on the id
        if max_id != min_id:
            return False
        assert max_id == min_id == new_id
        if new_id > self.remote_write_id or new_id < 0:
            self.remote_write_id = new_id
            return True
        return False

    def got_kill_signal(self):
        return self._got_kill_signal()

    def main(self):
        raise NotImplementedError

    def get_serial_number(self):
        return self.remote_write_id

    def _got_kill_signal(self):
        raise NotImplementedError


class _BoundSpoke(Spoke):
    """spoke.py:147-208."""

    def __init__(self, spbase_object, fullcomm, strata_comm, cylinder_comm, options=None):
        super().__init__(spbase_object, fullcomm, strata_comm, cylinder_comm, options)
        tp = spbase_object.options.get("trace_prefix") if hasattr(spbase_object, "options") else None
        if self.cylinder_rank == 0 and tp is not None:
            filen = tp + self.__class__.__name__ + ".csv"
            if os.path.exists(filen):
                raise RuntimeError(f"Spoke trace file {filen} already exists!")
            with open(filen, "w") as f:
                f.write("time,bound\n")
            self.trace_filen = filen
            self.start_time = spbase_object.start_time
        else:
            self.trace_filen = None
        self._new_locals = False
        self._bound = None
        self._locals = None

    def make_windows(self):
        self._make_windows(1, 2)
        self._locals = np.zeros(0 + 3)      # hub outer/inner bounds and kill signal
        self._bound = np.zeros(1 + 1)       # spoke bound + write id

    @property
    def bound(self):
        return self._bound[0]

    @bound.setter
    def bound(self, value):
        self._append_trace(value)
        self._bound[0] = value
        self.spoke_to_hub(self._bound)

    @property
    def hub_inner_bound(self):
        return self._locals[-2]

    @property
    def hub_outer_bound(self):
        return self._locals[-3]

    def _got_kill_signal(self):
        self._new_locals = self.spoke_from_hub(self._locals)
        return self.remote_write_id == -1

    def _append_trace(self, value):
        if self.cylinder_rank != 0 or self.trace_filen is None:
            return
        with open(self.trace_filen, "a") as f:
            f.write(f"{time.perf_counter() - self.start_time},{value}\n")


class _BoundNonantLenSpoke(_BoundSpoke):
    """spoke.py:211-236: the hub buffer holds one value per local nonant."""

    def make_windows(self):
        if not hasattr(self.opt, "local_scenarios"):
            raise RuntimeError("Provided SPBase object does not have local_scenarios attribute")
        if len(self.opt.local_scenarios) == 0:
            raise RuntimeError("Rank has zero local_scenarios")
        vbuflen = 2 + len(self.opt.local_scenarios) * self.opt.batch.nonant.N
        self._make_windows(1, vbuflen)
        self._locals = np.zeros(vbuflen + 1)
        self._bound = np.zeros(1 + 1)


class InnerBoundSpoke(_BoundSpoke):
    converger_spoke_types = (ConvergerSpokeType.INNER_BOUND,)
    converger_spoke_char = "I"


class OuterBoundSpoke(_BoundSpoke):
    converger_spoke_types = (ConvergerSpokeType.OUTER_BOUND,)
    converger_spoke_char = "O"


class _BoundWSpoke(_BoundNonantLenSpoke):
    @property
    def localWs(self):
        return self._locals[:-3]

    @property
    def new_Ws(self):
        return self._new_locals


class OuterBoundWSpoke(_BoundWSpoke):
    converger_spoke_types = (ConvergerSpokeType.OUTER_BOUND, ConvergerSpokeType.W_GETTER)
    converger_spoke_char = "O"


class _BoundNonantSpoke(_BoundNonantLenSpoke):
    @property
    def localnonants(self):
        return self._locals[:-3]

    @property
    def new_nonants(self):
        return self._new_locals


class InnerBoundNonantSpoke(_BoundNonantSpoke):
    """spoke.py:306-363.  The best-solution cache keeps the device solution
    (x of every local scenario) of the best incumbent."""
    converger_spoke_types = (ConvergerSpokeType.INNER_BOUND, ConvergerSpokeType.NONANT_GETTER)
    converger_spoke_char = "I"

    def __init__(self, spbase_object, fullcomm, strata_comm, cylinder_comm, options=None):
        super().__init__(spbase_object, fullcomm, strata_comm, cylinder_comm, options)
        self.is_minimizing = self.opt.is_minimizing
        self.best_inner_bound = math.inf if self.is_minimizing else -math.inf
        self.solver_options = None
        self.best_solution_cache = None

    def update_if_improving(self, candidate_inner_bound):
        if candidate_inner_bound is None:
            return False
        update = (candidate_inner_bound < self.best_inner_bound) if self.is_minimizing \
            else (self.best_inner_bound < candidate_inner_bound)
        if not update:
            return False
        self.best_inner_bound = candidate_inner_bound
        self.bound = candidate_inner_bound
        self._cache_best_solution()
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

    def _cache_best_solution(self):
        self.opt._settle()
        self.best_solution_cache = self.opt._x.clone()


class OuterBoundNonantSpoke(_BoundNonantSpoke):
    converger_spoke_types = (ConvergerSpokeType.OUTER_BOUND, ConvergerSpokeType.NONANT_GETTER)
    converger_spoke_char = "A"
