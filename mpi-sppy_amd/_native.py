"""ctypes binding of the phx C ABI (include/phx.h).

The product path loads ``libphx.so`` (built in-tree by ``build.py`` for
gfx950) and raises immediately if it is missing or no GPU is visible — there
is no CPU fallback.  The same wrapper can bind a library exporting the ABI
under another symbol prefix; the CPU test-suite uses that to bind the
test-only host emulation in ``tests/emu`` (never used by the product).
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# (PHX_LIB_PATH: an experiment's variant build; the product is the in-tree libphx.so)
LIB_PATH = os.environ.get("PHX_LIB_PATH") or os.path.join(_HERE, "libphx.so")

c_int32 = ctypes.c_int32
c_double = ctypes.c_double
c_void_p = ctypes.c_void_p
P_i32 = ctypes.POINTER(ctypes.c_int32)
P_f64 = ctypes.POINTER(ctypes.c_double)


class ProblemDesc(ctypes.Structure):
    _fields_ = [
        ("S", c_int32), ("n", c_int32), ("m", c_int32), ("nnz", c_int32),
        ("N", c_int32), ("nvar", c_int32),
        ("rowptr", c_void_p), ("colidx", c_void_p), ("kvar", c_void_p),
        ("Aconst", c_void_p), ("Avar", c_void_p),
        ("c", c_void_p), ("lb", c_void_p), ("ub", c_void_p),
        ("bl", c_void_p), ("bu", c_void_p),
        ("c_vary", c_int32), ("bnd_vary", c_int32), ("rhs_vary", c_int32),
        ("slot_col", c_void_p),
        ("lane_multi_theta", ctypes.c_double), ("lane_multi_rounds", c_int32),
    ]


class SolveOpts(ctypes.Structure):
    _fields_ = [
        ("max_iters", c_int32), ("check_every", c_int32), ("restart_max", c_int32),
        ("polish", c_int32), ("refine_steps", c_int32), ("warm_start", c_int32),
        ("polish_below", c_double), ("opt_tol", c_double), ("kkt_tol", c_double),
        ("reg", c_double),
        ("ipm_after", c_int32), ("ipm_max_it", c_int32), ("ipm_tol", c_double),
        ("lane_solver", c_int32), ("as_rounds", c_int32), ("warm_passes", c_int32),
        ("defer", c_int32), ("wg_warm", c_int32), ("sp", c_int32), ("sp_rounds", c_int32),
        ("seed_templates", c_int32), ("rescue_rounds", c_int32), ("lane_ipm_tol", c_double),
        ("wg_first", c_int32),
    ]


class SolveStats(ctypes.Structure):
    _fields_ = [
        ("pdhg_ms", c_double), ("polish_ms", c_double), ("ipm_ms", c_double), ("lane_ms", c_double),
        ("lane_warm_ms", c_double), ("lane_warm_list_ms", c_double),
        ("lane_iters", c_double), ("pdhg_launches", c_int32), ("total_iters", c_int32),
        ("lane_certified", c_int32), ("lane_warm_certified", c_int32), ("not_optimal", c_int32), ("stragglers", c_int32), ("jit", c_int32),
        ("lane_first_certified", c_int32), ("wg_certified", c_int32), ("wg_ms", c_double),
        ("sp_certified", c_int32), ("sp_warm_rounds", c_int32), ("sp_ipm_its", c_int32),
        ("sp_cold_rounds", c_int32), ("sp_refine", c_int32), ("sp_ms", c_double),
        ("infeasible", c_int32),
    ]


class TreeDesc(ctypes.Structure):
    _fields_ = [
        ("ntiles", c_int32),
        ("tile_s0", c_void_p), ("tile_s1", c_void_p), ("tile_slot", c_void_p),
        ("tile_nlen", c_void_p), ("tile_out", c_void_p),
        ("nnodes", c_int32),
        ("node_tile_ptr", c_void_p), ("node_off", c_void_p), ("node_nlen", c_void_p),
        ("NNS", c_int32), ("npart", c_int32), ("nnodes_cover", c_int32),
        ("node_key", c_void_p),
    ]


ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, c_void_p, c_void_p, ctypes.c_int64, c_void_p)


class IterkArgs(ctypes.Structure):
    _fields_ = [
        ("x", c_void_p), ("y", c_void_p), ("obj", c_void_p), ("status", c_void_p), ("iters", c_void_p),
        ("tree", ctypes.POINTER(TreeDesc)), ("prob_coeff", c_void_p), ("partial", c_void_p),
        ("node_sums", c_void_p), ("node_stage", c_void_p),
        ("xbar_idx", c_void_p), ("rho", c_void_p), ("W", c_void_p),
        ("nseg", c_int32), ("seg_s0_host", c_void_p), ("seg_s1_host", c_void_p), ("seg_sums", c_void_p),
        ("conv_counts_host", c_void_p), ("conv_R", c_int32), ("convthresh", c_double),
        ("max_iters", c_int32), ("depth", c_int32), ("timing", c_int32),
        ("allreduce", ALLREDUCE_FN), ("allreduce_user", c_void_p), ("node_stage_len", c_int32),
        ("iter0_obj", c_void_p), ("iter0_status", c_void_p),
        ("iter0_prob", c_void_p), ("iter0_expect", c_void_p), ("iter0_expect_host", c_void_p),
    ]


class IterkResult(ctypes.Structure):
    _fields_ = [
        ("iters", c_int32), ("converged", c_int32), ("conv", c_double), ("solves", c_int32),
        ("straggler_stops", c_int32), ("stragglers", c_int32), ("not_optimal", c_int32),
        ("warm_ms", c_double), ("warm_launches", c_int32), ("wall_ms", c_double), ("fused", c_int32),
        ("adopted", c_int32), ("adopted_stragglers", c_int32),
    ]


# every symbol of include/phx.h (tests check the library exports all of them)
SYMBOLS = [
    "create", "destroy", "last_error", "build_info", "set_problem", "set_bounds", "set_ph_terms",
    "solve", "solve_finish", "objective", "xbar", "update_w", "expect", "export_slots", "last_solve_stats", "jit_info",
    "iterk", "iterk_prepare", "comm_unique_id", "set_comm", "debug_spd_inverse",
]


class NativeError(RuntimeError):
    pass


class Lib:
    """Typed handle on a library exporting the phx ABI under ``prefix``."""

    def __init__(self, path=LIB_PATH, prefix="phx_"):
        if not os.path.exists(path):
            raise NativeError(
                "libphx not found at %s — build it first (python -c 'import __graft_entry__ as g; "
                "g.build()'); the engine has no CPU fallback" % path)
        self.path = path
        self.prefix = prefix
        self.lib = ctypes.CDLL(path)
        L = self.lib

        def fn(name, res, args):
            f = getattr(L, prefix + name)
            f.restype = res
            f.argtypes = args
            return f

        self.create = fn("create", ctypes.c_int, [c_int32, ctypes.POINTER(c_void_p)])
        self.destroy = fn("destroy", ctypes.c_int, [c_void_p])
        self.last_error = fn("last_error", ctypes.c_char_p, [c_void_p])
        self.build_info = fn("build_info", ctypes.c_char_p, [])
        self.set_problem = fn("set_problem", ctypes.c_int, [c_void_p, ctypes.POINTER(ProblemDesc)])
        self.set_bounds = fn("set_bounds", ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_void_p])
        self.set_ph_terms = fn("set_ph_terms", ctypes.c_int,
                               [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_void_p])
        self.solve = fn("solve", ctypes.c_int,
                        [c_void_p, ctypes.POINTER(SolveOpts), c_void_p, c_void_p, c_void_p, c_void_p,
                         c_void_p, P_i32, c_void_p])
        self.solve_finish = fn("solve_finish", ctypes.c_int, [c_void_p, P_i32, P_i32])
        self.objective = fn("objective", ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_void_p])
        self.xbar = fn("xbar", ctypes.c_int,
                       [c_void_p, ctypes.POINTER(TreeDesc), c_void_p, c_void_p, c_void_p, c_void_p, c_void_p])
        self.update_w = fn("update_w", ctypes.c_int,
                           [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_void_p,
                            c_int32, P_i32, P_i32, c_void_p, c_void_p])
        self.expect = fn("expect", ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p])
        self.export_slots = fn("export_slots", ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_void_p])
        self.last_solve_stats = fn("last_solve_stats", ctypes.c_int, [c_void_p, ctypes.POINTER(SolveStats)])
        self.jit_info = fn("jit_info", ctypes.c_char_p, [c_void_p])
        self.iterk = fn("iterk", ctypes.c_int, [c_void_p, ctypes.POINTER(SolveOpts), ctypes.POINTER(IterkArgs),
                                                ctypes.POINTER(IterkResult), c_void_p])
        self.iterk_prepare = fn("iterk_prepare", ctypes.c_int, [c_void_p, ctypes.POINTER(IterkArgs)])
        self.comm_unique_id = fn("comm_unique_id", ctypes.c_int, [c_void_p])
        self.set_comm = fn("set_comm", ctypes.c_int, [c_void_p, c_void_p, c_int32, c_int32])
        self.debug_spd_inverse = fn("debug_spd_inverse", ctypes.c_int, [c_void_p, c_int32, c_void_p])

    def check(self, ctx, rc, what):
        if rc != 0:
            msg = self.last_error(ctx) if ctx else None
            raise NativeError("%s%s failed (rc=%d): %s" % (self.prefix, what, rc,
                                                          msg.decode() if msg else "?"))


_LIB = None


def load():
    """The product library (cached).  Raises NativeError if unavailable."""
    global _LIB
    if _LIB is None:
        _LIB = Lib(LIB_PATH, "phx_")
    return _LIB
