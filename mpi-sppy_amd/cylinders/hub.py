"""The hub: the cylinder that runs the PH algorithm, publishes W / nonants to
the spokes and collects their bounds (the role of mpisppy/cylinders/hub.py:23-598
-- ``Hub``, ``PHHub`` -- restructured around three pieces):

* ``BoundBook``  the best inner and outer bounds of a minimisation or
  maximisation, which spoke improved them last, the gaps and the stall count;
* ``_Link``      per spoke: its roles (from its class's
  ``converger_spoke_types``), the hub's ``Outbox`` to it and the ``Inbox`` of
  its bound (cylinders/channel.py);
* ``Hub``        the handshake, publishing one payload per kind to every spoke
  that wants it (W, nonants, bounds only), collecting bounds, the termination
  rule (rel_gap / abs_gap / max_stalled_iters options) and the screen trace.

``PHHub`` is what PHBase sees as ``spcomm``: ``sync()`` after Iter0 and every
iteration, ``is_converged()``.  The W / nonant payloads are formed on the
device (one transpose kernel + one D2H of S*N doubles: ``_populate_W_cache`` /
``nonant_values``) and written into the hub's node-local windows.
"""
import logging
from math import inf, isfinite

import numpy as np

from .channel import Inbox, Outbox
from .spcommunicator import SPCommunicator, window_lengths
from .spoke import ConvergerSpokeType

logger = logging.getLogger("mpisppy_amd.cylinders.Hub")


def global_toc(msg, cond=True):
    from ..spbase import _global_toc
    _global_toc(msg, cond)


class BoundBook:
    """Best bounds so far, in the problem's sense."""

    def __init__(self, minimizing):
        self.minimizing = minimizing
        self.inner = inf if minimizing else -inf      # best incumbent
        self.outer = -inf if minimizing else inf      # best bound
        self.inner_mark = self.outer_mark = None      # char of the last improvement (screen trace)
        self.inner_src = self.outer_src = None        # spoke index of it (0: the hub)
        self._best_gap = inf
        self.stalled = 0

    def offer_inner(self, value, mark, src):
        better = value < self.inner if self.minimizing else value > self.inner
        if better:
            self.inner, self.inner_mark, self.inner_src = value, mark, src
        return better

    def offer_outer(self, value, mark, src):
        better = value > self.outer if self.minimizing else value < self.outer
        if better:
            self.outer, self.outer_mark, self.outer_src = value, mark, src
        return better

    def gaps(self):
        """(absolute, relative) gap; relative is inf while undefined."""
        ag = self.inner - self.outer if self.minimizing else self.outer - self.inner
        ok = not np.isnan(ag) and isfinite(ag) and not np.isnan(self.outer) and self.outer != 0
        return ag, (ag / abs(self.outer) if ok else inf)

    def note_gap(self):
        """Stall counter: iterations since the absolute gap last shrank."""
        ag = self.gaps()[0]
        if ag < self._best_gap:
            self._best_gap, self.stalled = ag, 0
        else:
            self.stalled += 1
        return self.stalled

    def marks(self):
        o = self.outer_mark or " "
        i = self.inner_mark or " "
        return o + " " + i

    def clear_marks(self):
        self.inner_mark = self.outer_mark = None


class _Link:
    """The hub's view of one spoke."""

    def __init__(self, index, spoke_class, out, inbox):
        self.index = index                            # its strata rank
        roles = set(getattr(spoke_class, "converger_spoke_types", ()))
        unknown = roles - set(ConvergerSpokeType)
        if unknown:
            raise RuntimeError("Unrecognized converger_spoke_type %s" % unknown)
        self.outer = ConvergerSpokeType.OUTER_BOUND in roles
        self.inner = ConvergerSpokeType.INNER_BOUND in roles
        self.wants_W = ConvergerSpokeType.W_GETTER in roles
        self.wants_nonants = ConvergerSpokeType.NONANT_GETTER in roles
        self.mark = getattr(spoke_class, "converger_spoke_char", "?")
        self.out = out                                # Outbox: hub -> spoke
        self.inbox = inbox                            # Inbox: spoke -> hub
        self.recv = np.zeros(inbox.length + 1)

    @property
    def kind(self):
        return "W" if self.wants_W else ("nonants" if self.wants_nonants else "bounds")


class Hub(SPCommunicator):
    def __init__(self, spbase_object, fullcomm, strata_comm, cylinder_comm, spokes, options=None):
        super().__init__(spbase_object, fullcomm, strata_comm, cylinder_comm, options=options)
        if len(spokes) != self.n_spokes:
            raise RuntimeError("%d spoke descriptions for %d spoke ranks" % (len(spokes), self.n_spokes))
        self.spokes = spokes
        self.links = []
        self.book = BoundBook(self.opt.is_minimizing)
        self.print_init = True
        self._payloads = {}                           # kind -> send buffer

    # ---- the reference's attribute names
    @property
    def BestInnerBound(self):
        return self.book.inner

    @BestInnerBound.setter
    def BestInnerBound(self, v):
        self.book.inner = v

    @property
    def BestOuterBound(self):
        return self.book.outer

    @BestOuterBound.setter
    def BestOuterBound(self, v):
        self.book.outer = v

    @property
    def last_ib_idx(self):
        return self.book.inner_src

    @property
    def last_ob_idx(self):
        return self.book.outer_src

    @property
    def local_write_ids(self):
        return np.array([ln.out.write_id for ln in self.links], dtype=np.int64)

    @property
    def remote_write_ids(self):
        return np.array([ln.inbox.read_id for ln in self.links], dtype=np.int64)

    def _with(self, pred):
        return [ln for ln in self.links if pred(ln)]

    @property
    def has_outerbound_spokes(self):
        return bool(self._with(lambda ln: ln.outer))

    @property
    def has_innerbound_spokes(self):
        return bool(self._with(lambda ln: ln.inner))

    # ---- setup
    def make_windows(self):
        """Handshake: every spoke announces (its own buffer length, the length
        it wants from the hub); one window per spoke."""
        if self._windows_constructed:
            return
        ann = self.strata_comm.allgather_object(None)[1:]
        own = [int(a[0]) for a in ann]
        wanted = [int(a[1]) for a in ann]
        self._make_windows_from_lengths(window_lengths(wanted, own))
        self.links = [_Link(i + 1, self.spokes[i]["spoke_class"],
                            Outbox(self.windows[i], 0, wanted[i], self.cylinder_comm),
                            Inbox(self.windows[i], i + 1, own[i], self.cylinder_comm))
                      for i in range(self.n_spokes)]

    def setup_hub(self):
        if not self._windows_constructed:
            raise RuntimeError("Cannot call setup_hub before memory windows are constructed")
        for ln in self.links:
            if ln.outer and ln.inner:
                raise RuntimeError("A Spoke providing both inner and outer bounds is currently unsupported")
            if ln.wants_W and ln.wants_nonants:
                raise RuntimeError("A Spoke needing both Ws and nonants is currently unsupported")
        # one send buffer per payload kind; every receiver of a kind must want
        # the same length
        for ln in self.links:
            buf = self._payloads.get(ln.kind)
            if buf is None:
                self._payloads[ln.kind] = np.zeros(ln.out.length + 1)
            elif len(buf) != ln.out.length + 1:
                raise RuntimeError("%s buffers of the spokes disagree on size" % ln.kind)
        if ("bounds" in self._payloads and len(self._payloads["bounds"]) != 3):
            raise RuntimeError("a bounds-only spoke must want exactly the two bounds")
        if not self.has_outerbound_spokes:
            logger.warning("No OuterBound Spokes defined, this converger will not cause the hub to terminate")
        if not self.has_innerbound_spokes:
            logger.warning("No InnerBound Spokes defined, this converger will not cause the hub to terminate")

    # ---- traffic
    def _fill(self, kind, buf):
        """The payload part of a send buffer (the bounds are added after)."""
        raise NotImplementedError

    def _publish(self, only=None):
        for kind, buf in self._payloads.items():
            if only is not None and kind != only:
                continue
            self._fill(kind, buf)
            buf[-3], buf[-2] = self.book.outer, self.book.inner
            for ln in self.links:
                if ln.kind == kind:
                    ln.out.publish(buf)

    def _collect(self):
        for ln in self.links:
            if (ln.outer or ln.inner) and ln.inbox.poll(ln.recv):
                offer = self.book.offer_outer if ln.outer else self.book.offer_inner
                offer(ln.recv[0], ln.mark, ln.index)

    def send_terminate(self):
        for ln in self.links:
            ln.out.kill()

    # ---- termination and reporting
    def compute_gaps(self):
        return self.book.gaps()

    def current_iteration(self):
        raise NotImplementedError

    def screen_trace(self):
        show = self.options.get("display_progress", True)
        if self.print_init:
            global_toc("%5s  %3s  %14s  %14s  %12s  %14s" % ("Iter.", "", "Best Bound", "Best Incumbent",
                                                              "Rel. Gap", "Abs. Gap"), show)
            self.print_init = False
        ag, rg = self.book.gaps()
        global_toc("%5d  %3s  %14.4f  %14.4f  %11.3f%%  %14.4f"
                   % (self.current_iteration(), self.book.marks(), self.book.outer, self.book.inner, rg * 100, ag),
                   show)
        self.book.clear_marks()

    def determine_termination(self):
        """True once the gap is within the rel_gap / abs_gap options or it has
        not shrunk for max_stalled_iters checks."""
        o = self.options or {}
        keys = [k for k in ("rel_gap", "abs_gap", "max_stalled_iters") if k in o]
        if not keys:
            return False
        ag, rg = self.book.gaps()
        reasons = []
        if "abs_gap" in o and ag <= o["abs_gap"]:
            reasons.append("inter-cylinder absolute gap %12.4f" % ag)
        if "rel_gap" in o and rg <= o["rel_gap"]:
            reasons.append("inter-cylinder relative gap %12.3f%%" % (rg * 100))
        if "max_stalled_iters" in o and self.book.note_gap() >= o["max_stalled_iters"]:
            reasons.append("max-stalled-iters %d" % self.book.stalled)
        for r in reasons:
            global_toc("Terminating based on " + r)
        return bool(reasons)

    def hub_finalize(self):
        """The spokes' last bounds, then the final trace line."""
        self._collect()
        if self.global_rank == 0:
            self.print_init = True
            global_toc("Statistics at termination", True)
            self.screen_trace()


class PHHub(Hub):
    """The PH algorithm's hub (``spcomm`` of PHBase)."""

    def _fill(self, kind, buf):
        if kind == "W":
            self.opt._populate_W_cache(buf, padding=3)
        elif kind == "nonants":
            self.opt._save_nonants()
            flat = self.opt.nonant_values().ravel()
            buf[:len(flat)] = flat

    def sync(self):
        """After Iter0 and every PH iteration: publish each payload kind some
        spoke wants (send_ws / send_nonants / send_boundsout), then collect."""
        for kind, send in (("W", self.send_ws), ("nonants", self.send_nonants), ("bounds", self.send_boundsout)):
            if kind in self._payloads:
                send()
        self._collect()

    def sync_with_spokes(self):
        self.sync()

    def send_ws(self):
        self._publish("W")

    def send_nonants(self):
        self._publish("nonants")

    def send_boundsout(self):
        self._publish("bounds")

    # (the reference's names of the three send buffers)
    @property
    def w_send_buffer(self):
        return self._payloads.get("W")

    @property
    def nonant_send_buffer(self):
        return self._payloads.get("nonants")

    @property
    def boundsout_send_buffer(self):
        return self._payloads.get("bounds")

    def is_converged(self):
        first = self.opt._PHIter == 1
        if first:
            # Iter0's trivial bound is the first outer bound (mark "*": the hub's own)
            self.book.offer_outer(self.opt.trivial_bound, "*", 0)
        if not self.has_innerbound_spokes:
            if first:
                logger.warning("PHHub cannot compute convergence without inner bound spokes.")
            if self.global_rank == 0:
                self.screen_trace()
            return False
        if first and not self.has_outerbound_spokes:
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
