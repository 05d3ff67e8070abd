"""Hub side of the hub-and-spoke system (cylinders/hub.py:23-598).

``Hub`` keeps the reference's bookkeeping (best inner/outer bounds, gaps,
termination by rel_gap / abs_gap / max_stalled_iters, the screen trace) and its
wire format: per spoke one flat fp64 buffer ``[payload | outer, inner,
write_id]`` (hub.py:281-285), a write id incremented per put, agreement on it
across the cylinder's ranks before a value counts as new (hub.py:396-436), and
the kill signal ``write_id = -1`` (hub.py:438-450).  ``PHHub`` is the PH
opt-object's spcomm: ``sync()`` after Iter0 and every iteration sends W
(``send_ws``, hub.py:590-598) and/or nonants (``send_nonants``, :562-577) and
receives the spokes' bounds; ``is_converged()`` is hub.py:519-547.

The flat W / nonant payloads are formed on the device (``_populate_W_cache`` /
``_save_nonants``: one transpose kernel + one D2H of S*N doubles) and written
into the hub's node-local window (``spwindow.SPWindow``).
"""
import logging
from math import inf

import numpy as np

from .spcommunicator import SPCommunicator
from .spoke import ConvergerSpokeType

logger = logging.getLogger("mpisppy_amd.cylinders.Hub")


def global_toc(msg, cond=True):
    from ..spbase import _global_toc
    _global_toc(msg, cond)


class Hub(SPCommunicator):
    def __init__(self, spbase_object, fullcomm, strata_comm, cylinder_comm, spokes, options=None):
        super().__init__(spbase_object, fullcomm, strata_comm, cylinder_comm, options=options)
        assert len(spokes) == self.n_spokes
        self.local_write_ids = np.zeros(self.n_spokes, dtype=np.int64)
        self.remote_write_ids = np.zeros(self.n_spokes, dtype=np.int64)
        self.local_lengths = np.zeros(self.n_spokes, dtype=np.int64)
        self.remote_lengths = np.zeros(self.n_spokes, dtype=np.int64)
        self.spokes = spokes
        self.print_init = True
        self.latest_ib_char = None
        self.latest_ob_char = None
        self.last_ib_idx = None
        self.last_ob_idx = None
        self.stalled_iter_cnt = 0
        self.last_gap = float("inf")

    def setup_hub(self):
        raise NotImplementedError

    def current_iteration(self):
        raise NotImplementedError

    def clear_latest_chars(self):
        self.latest_ib_char = None
        self.latest_ob_char = None

    def compute_gaps(self):
        """hub.py:77-98."""
        if self.opt.is_minimizing:
            abs_gap = self.BestInnerBound - self.BestOuterBound
        else:
            abs_gap = self.BestOuterBound - self.BestInnerBound
        if (not np.isnan(abs_gap) and abs_gap not in (inf, -inf)
                and not np.isnan(self.BestOuterBound) and self.BestOuterBound != 0):
            rel_gap = abs_gap / abs(self.BestOuterBound)
        else:
            rel_gap = float("inf")
        return abs_gap, rel_gap

    def get_update_string(self):
        if self.latest_ib_char is None and self.latest_ob_char is None:
            return "   "
        if self.latest_ib_char is None:
            return self.latest_ob_char + "  "
        if self.latest_ob_char is None:
            return "  " + self.latest_ib_char
        return self.latest_ob_char + " " + self.latest_ib_char

    def screen_trace(self):
        current_iteration = self.current_iteration()
        abs_gap, rel_gap = self.compute_gaps()
        if self.print_init:
            row = (f'{"Iter.":>5s}  {"   "}  {"Best Bound":>14s}  {"Best Incumbent":>14s}  {"Rel. Gap":>12s}  '
                   f'{"Abs. Gap":>14s}')
            global_toc(row, self.options.get("display_progress", True))
            self.print_init = False
        row = (f"{current_iteration:5d}  {self.get_update_string()}  {self.BestOuterBound:14.4f}  "
               f"{self.BestInnerBound:14.4f}  {rel_gap * 100:12.3f}%  {abs_gap:14.4f}")
        global_toc(row, self.options.get("display_progress", True))
        self.clear_latest_chars()

    def determine_termination(self):
        """hub.py:125-161."""
        o = self.options
        if o is None or ("rel_gap" not in o and "abs_gap" not in o and "max_stalled_iters" not in o):
            return False
        abs_gap, rel_gap = self.compute_gaps()
        rel_ok = "rel_gap" in o and rel_gap <= o["rel_gap"]
        abs_ok = "abs_gap" in o and abs_gap <= o["abs_gap"]
        stalled = False
        if "max_stalled_iters" in o:
            if abs_gap < self.last_gap:
                self.last_gap = abs_gap
                self.stalled_iter_cnt = 0
            else:
                self.stalled_iter_cnt += 1
                stalled = self.stalled_iter_cnt >= o["max_stalled_iters"]
        if abs_ok:
            global_toc(f"Terminating based on inter-cylinder absolute gap {abs_gap:12.4f}")
        if rel_ok:
            global_toc(f"Terminating based on inter-cylinder relative gap {rel_gap * 100:12.3f}%")
        if stalled:
            global_toc(f"Terminating based on max-stalled-iters {self.stalled_iter_cnt}")
        return abs_ok or rel_ok or stalled

    def hub_finalize(self):
        if self.has_outerbound_spokes:
            self.receive_outerbounds()
        if self.has_innerbound_spokes:
            self.receive_innerbounds()
        if self.global_rank == 0:
            self.print_init = True
            global_toc("Statistics at termination", True)
            self.screen_trace()

    def receive_innerbounds(self):
        for idx in sorted(self.innerbound_spoke_indices):
            if self.hub_from_spoke(self.innerbound_receive_buffers[idx], idx):
                self.BestInnerBound = self.InnerBoundUpdate(self.innerbound_receive_buffers[idx][0], idx)

    def receive_outerbounds(self):
        for idx in sorted(self.outerbound_spoke_indices):
            if self.hub_from_spoke(self.outerbound_receive_buffers[idx], idx):
                self.BestOuterBound = self.OuterBoundUpdate(self.outerbound_receive_buffers[idx][0], idx)

    def OuterBoundUpdate(self, new_bound, idx=None, char="*"):
        current = self.BestOuterBound
        if self._outer_bound_update(new_bound, current):
            if idx is None:
                self.latest_ob_char = char
                self.last_ob_idx = 0
            else:
                self.latest_ob_char = self.outerbound_spoke_chars[idx]
                self.last_ob_idx = idx
            return new_bound
        return current

    def InnerBoundUpdate(self, new_bound, idx=None, char="*"):
        current = self.BestInnerBound
        if self._inner_bound_update(new_bound, current):
            if idx is None:
                self.latest_ib_char = char
                self.last_ib_idx = 0
            else:
                self.latest_ib_char = self.innerbound_spoke_chars[idx]
                self.last_ib_idx = idx
            return new_bound
        return current

    def initialize_bound_values(self):
        if self.opt.is_minimizing:
            self.BestInnerBound, self.BestOuterBound = inf, -inf
            self._inner_bound_update = lambda new, old: new < old
            self._outer_bound_update = lambda new, old: new > old
        else:
            self.BestInnerBound, self.BestOuterBound = -inf, inf
            self._inner_bound_update = lambda new, old: new > old
            self._outer_bound_update = lambda new, old: new < old

    def initialize_outer_bound_buffers(self):
        self.outerbound_receive_buffers = {idx: np.zeros(self.remote_lengths[idx - 1] + 1)
                                           for idx in self.outerbound_spoke_indices}

    def initialize_inner_bound_buffers(self):
        self.innerbound_receive_buffers = {idx: np.zeros(self.remote_lengths[idx - 1] + 1)
                                           for idx in self.innerbound_spoke_indices}

    def initialize_nonants(self):
        self.nonant_send_buffer = None
        for idx in self.nonant_spoke_indices:
            if self.nonant_send_buffer is None:
                self.nonant_send_buffer = np.zeros(self.local_lengths[idx - 1] + 1)
            elif self.local_lengths[idx - 1] + 1 != len(self.nonant_send_buffer):
                raise RuntimeError("Nonant buffers disagree on size")

    def initialize_boundsout(self):
        self.boundsout_send_buffer = None
        for idx in self.bounds_only_indices:
            if self.boundsout_send_buffer is None:
                self.boundsout_send_buffer = np.zeros(self.local_lengths[idx - 1] + 1)
            if self.local_lengths[idx - 1] != 2:
                raise RuntimeError("bounds only local length buffers must be 2 (bounds). "
                                   f"Currently {self.local_lengths[idx - 1]}")

    def _populate_boundsout_cache(self, buf):
        buf[-3] = self.BestOuterBound
        buf[-2] = self.BestInnerBound

    def send_boundsout(self):
        self._populate_boundsout_cache(self.boundsout_send_buffer)
        for idx in sorted(self.bounds_only_indices):
            self.hub_to_spoke(self.boundsout_send_buffer, idx)

    def initialize_spoke_indices(self):
        """hub.py:297-343."""
        self.outerbound_spoke_indices = set()
        self.innerbound_spoke_indices = set()
        self.nonant_spoke_indices = set()
        self.w_spoke_indices = set()
        self.outerbound_spoke_chars = dict()
        self.innerbound_spoke_chars = dict()
        for i, spoke in enumerate(self.spokes):
            cls = spoke["spoke_class"]
            for cst in getattr(cls, "converger_spoke_types", ()):
                if cst == ConvergerSpokeType.OUTER_BOUND:
                    self.outerbound_spoke_indices.add(i + 1)
                    self.outerbound_spoke_chars[i + 1] = cls.converger_spoke_char
                elif cst == ConvergerSpokeType.INNER_BOUND:
                    self.innerbound_spoke_indices.add(i + 1)
                    self.innerbound_spoke_chars[i + 1] = cls.converger_spoke_char
                elif cst == ConvergerSpokeType.W_GETTER:
                    self.w_spoke_indices.add(i + 1)
                elif cst == ConvergerSpokeType.NONANT_GETTER:
                    self.nonant_spoke_indices.add(i + 1)
                else:
                    raise RuntimeError(f"Unrecognized converger_spoke_type {cst}")
        self.bounds_only_indices = ((self.outerbound_spoke_indices | self.innerbound_spoke_indices)
                                    - (self.w_spoke_indices | self.nonant_spoke_indices))
        self.has_outerbound_spokes = len(self.outerbound_spoke_indices) > 0
        self.has_innerbound_spokes = len(self.innerbound_spoke_indices) > 0
        self.has_nonant_spokes = len(self.nonant_spoke_indices) > 0
        self.has_w_spokes = len(self.w_spoke_indices) > 0
        self.has_bounds_only_spokes = len(self.bounds_only_indices) > 0

    def make_windows(self):
        """The spokes announce (their buffer length, the length they want from
        the hub) (hub.py:345-368 / spoke.py:34-58); one window per spoke."""
        if self._windows_constructed:
            return
        pairs = self.strata_comm.allgather_object(None)
        for i in range(self.n_spokes):
            self.remote_lengths[i] = int(pairs[i + 1][0])
            self.local_lengths[i] = int(pairs[i + 1][1])
        self._make_windows_from_lengths(_window_lengths(self.n_spokes, self.local_lengths, self.remote_lengths))

    def hub_to_spoke(self, values, spoke_strata_rank):
        """hub.py:370-394: write id += 1, one put into the hub's own buffer."""
        expected = self.local_lengths[spoke_strata_rank - 1] + 1
        if len(values) != expected:
            raise RuntimeError(f"Attempting to put array of length {len(values)} "
                               f"into local buffer of length {expected}")
        # so the spoke ranks all get the same write_id at approximately the same time
        self.cylinder_comm.Barrier()
        self.local_write_ids[spoke_strata_rank - 1] += 1
        values[-1] = self.local_write_ids[spoke_strata_rank - 1]
        self.windows[spoke_strata_rank - 1].put(values)

    def hub_from_spoke(self, values, spoke_num):
        """hub.py:396-436: the value is new only if every cylinder rank read
        the same write id and it is newer than the last one (or negative)."""
        expected = self.remote_lengths[spoke_num - 1] + 1
        if len(values) != expected:
            raise RuntimeError(f"Hub trying to get buffer of length {expected} "
                               f"from spoke, but provided buffer has length {len(values)}.")
        self.cylinder_comm.Barrier()
        self.windows[spoke_num - 1].get(spoke_num, values)
        new_id = int(values[-1])
        sum_ids = self.cylinder_comm.allreduce_np(np.array([new_id], dtype=np.int64), op="sum")
        if new_id != sum_ids[0] / self.cylinder_comm.Get_size():
            return False
        if new_id > self.remote_write_ids[spoke_num - 1] or new_id < 0:
            self.remote_write_ids[spoke_num - 1] = new_id
            return True
        return False

    def send_terminate(self):
        """hub.py:438-450: zeros with write id -1 into every spoke's window."""
        for rank in range(1, self.n_spokes + 1):
            dummies = np.zeros(self.local_lengths[rank - 1] + 1)
            dummies[-1] = -1
            self.windows[rank - 1].put(dummies)


def _window_lengths(n_spokes, hub_lengths, spoke_lengths):
    """Window i (spoke i+1): the hub owns hub_lengths[i] doubles (hub ->
    spoke), spoke i+1 owns spoke_lengths[i] (spoke -> hub), the others none."""
    out = []
    for i in range(n_spokes):
        ln = [0] * (n_spokes + 1)
        ln[0] = int(hub_lengths[i])
        ln[i + 1] = int(spoke_lengths[i])
        out.append(ln)
    return out


class PHHub(Hub):
    def setup_hub(self):
        """hub.py:454-499."""
        if not self._windows_constructed:
            raise RuntimeError("Cannot call setup_hub before memory windows are constructed")
        self.initialize_spoke_indices()
        self.initialize_bound_values()
        if self.has_outerbound_spokes:
            self.initialize_outer_bound_buffers()
        if self.has_innerbound_spokes:
            self.initialize_inner_bound_buffers()
        if self.has_w_spokes:
            self.initialize_ws()
        if self.has_nonant_spokes:
            self.initialize_nonants()
        if self.has_bounds_only_spokes:
            self.initialize_boundsout()
        if len(self.outerbound_spoke_indices & self.innerbound_spoke_indices) > 0:
            raise RuntimeError("A Spoke providing both inner and outer bounds is currently unsupported")
        if len(self.w_spoke_indices & self.nonant_spoke_indices) > 0:
            raise RuntimeError("A Spoke needing both Ws and nonants is currently unsupported")
        if not self.has_outerbound_spokes:
            logger.warning("No OuterBound Spokes defined, this converger will not cause the hub to terminate")
        if not self.has_innerbound_spokes:
            logger.warning("No InnerBound Spokes defined, this converger will not cause the hub to terminate")

    def sync(self):
        """hub.py:501-514."""
        if self.has_w_spokes:
            self.send_ws()
        if self.has_nonant_spokes:
            self.send_nonants()
        if self.has_bounds_only_spokes:
            self.send_boundsout()
        if self.has_outerbound_spokes:
            self.receive_outerbounds()
        if self.has_innerbound_spokes:
            self.receive_innerbounds()

    def sync_with_spokes(self):
        self.sync()

    def is_converged(self):
        """hub.py:519-547."""
        if self.opt._PHIter == 1:
            self.BestOuterBound = self.OuterBoundUpdate(self.opt.trivial_bound)
        if not self.has_innerbound_spokes:
            if self.opt._PHIter == 1:
                logger.warning("PHHub cannot compute convergence without inner bound spokes.")
            if self.global_rank == 0:
                self.screen_trace()
            return False
        if not self.has_outerbound_spokes and self.opt._PHIter == 1:
            global_toc("Without outer bound spokes, no progress will be made on the Best Bound")
        if self.global_rank == 0:
            self.screen_trace()
        return self.determine_termination()

    def current_iteration(self):
        return self.opt._PHIter

    def main(self):
        self.opt.ph_main(finalize=False)

    def finalize(self):
        return self.opt.post_loops(self.opt.extensions)

    def send_nonants(self):
        """hub.py:562-577: the local scenarios' nonants, scenario-major."""
        self.opt._save_nonants()
        buf = self.nonant_send_buffer
        flat = self.opt.nonant_values().ravel()
        buf[:len(flat)] = flat
        self._populate_boundsout_cache(buf)
        for idx in sorted(self.nonant_spoke_indices):
            self.hub_to_spoke(buf, idx)

    def initialize_ws(self):
        self.w_send_buffer = None
        for idx in self.w_spoke_indices:
            if self.w_send_buffer is None:
                self.w_send_buffer = np.zeros(self.local_lengths[idx - 1] + 1)
            elif self.local_lengths[idx - 1] + 1 != len(self.w_send_buffer):
                raise RuntimeError("W buffers disagree on size")

    def send_ws(self):
        """hub.py:590-598."""
        self.opt._populate_W_cache(self.w_send_buffer, padding=3)
        self._populate_boundsout_cache(self.w_send_buffer)
        for idx in sorted(self.w_spoke_indices):
            self.hub_to_spoke(self.w_send_buffer, idx)
