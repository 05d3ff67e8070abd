"""Host wall-clock timeline of the bench's timed region (Iter0 + K iterations,
farmer 100k): every PHBase/SPOpt/SPBase method call and native ABI call, with
its start/end relative to Iter0's start (second of two runs)."""
import functools
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import mpisppy_amd  # noqa: E402,F401
from mpisppy_amd import phbase, spopt, spbase, _native  # noqa: E402
from mpisppy_amd.examples import farmer  # noqa: E402

REC = []
DEPTH = [0]


def wrap(name, f):
    @functools.wraps(f)
    def g(*a, **k):
        d = DEPTH[0]
        DEPTH[0] += 1
        t0 = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            DEPTH[0] -= 1
            REC.append((t0, time.perf_counter(), d, name))
    return g


for cls in (phbase.PHBase, spopt.SPOpt, spbase.SPBase):
    for nm, f in list(vars(cls).items()):
        if callable(f) and not nm.startswith("__") and not isinstance(f, (staticmethod, classmethod, property)):
            setattr(cls, nm, wrap(cls.__name__ + "." + nm, f))
_orig_init = _native.Lib.__init__


def _init(self, *a, **k):
    _orig_init(self, *a, **k)
    for nm in _native.SYMBOLS:
        f = getattr(self, nm, None)
        if f is not None:
            setattr(self, nm, wrap("abi." + nm, f))


_native.Lib.__init__ = _init
import gc  # noqa: E402
GC = []
gc.callbacks.append(lambda phase, info: GC.append((time.perf_counter(), phase, info.get("generation"))))
if os.environ.get("GC_FREEZE"):
    gc.collect()
    gc.freeze()
S = int(os.environ.get("SCENS", "100000"))
w = {"names": farmer.scenario_names_creator, "creator": farmer.scenario_creator,
     "kw": lambda S, cm: {"num_scens": S, "crops_multiplier": cm}, "nodes": None}
dev = bench.Dev(os.environ.get("DEV", "cuda"))
for rep in range(2):
    ph = bench.make_ph(w, S, 1, 1.0, {}, 20, dev)
    dev.sync()
    REC.clear()
    GC.clear()
    T = bench.timed_run(ph, 20, dev)
    print("run", rep, "T, T_iter0, T_iterk (ms):", ["%.3f" % (1e3 * v) for v in T])
    del ph
t_first = min(r[0] for r in REC if r[3].endswith("Iter0"))
for t0, t1, d, name in sorted(REC):
    if t0 >= t_first - 1e-3:
        print("%9.1f %9.1f  %s%s" % ((t0 - t_first) * 1e6, (t1 - t0) * 1e6, "  " * d, name))
gcs = [g for g in GC if g[0] >= t_first - 1e-3]
for (ta, pa, ga), (tb, pb, gb) in zip(gcs[::2], gcs[1::2]):
    print("%9.1f %9.1f  gc generation %s" % ((ta - t_first) * 1e6, (tb - ta) * 1e6, ga))
