"""Shared helpers for the parity tests (run the engine and the oracle side by side)."""
import numpy as np

import mpisppy_amd  # noqa: F401
from mpisppy_amd.opt.ph import PH
from oracle import models as om, ph as oph


def ph_options(iters, rho=1.0, convthresh=1e-10, solver=None):
    return {"solver_name": "phx", "PHIterLimit": iters, "defaultPHrho": rho, "convthresh": convthresh,
            "verbose": False, "display_progress": False,
            "iter0_solver_options": dict(solver or {}), "iterk_solver_options": dict(solver or {})}


def rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.max(np.abs(a - b) / np.maximum(1.0, np.abs(b)))) if a.size else 0.0


def run_engine(creator, names, kwargs, iters, rho=1.0, lib=None, device=None, all_nodenames=None,
               options=None, mpicomm=None):
    opts = ph_options(iters, rho)
    if options:
        opts.update(options)
    ph = PH(opts, names, creator, scenario_creator_kwargs=kwargs, all_nodenames=all_nodenames,
            mpicomm=mpicomm, _native_lib=lib, _device=device)
    conv, Eobj, tb = ph.ph_main()
    return ph, conv, Eobj, tb


REF_XBAR = np.array([96.88717449844287, 274.2239371483933, 128.88888831920772])
REF_W = np.array([[-16.10425295139681, 70.84705093609978, -54.742797934166234],
                  [-41.104251445950844, 89.57647412029155, -48.47222265026873],
                  [57.20850439734766, -160.42352505639107, 103.21502058443501]])


def oracle_continue_from(ph_iter0, scens, iters, rho=1.0, convthresh=1e-10):
    """The oracle's PH iterations 1..iters started from the engine's Iter0 point
    (degenerate Iter0 LPs may have several optimal vertices; from iteration 1 on the
    prox term makes each subproblem's nonant optimum unique, so the trajectories must
    agree).  ph_iter0: an engine run with PHIterLimit = 0."""
    o = oph.OraclePH(scens, rho=rho)
    x = ph_iter0._host("x")
    for k in range(len(scens)):
        o.x[k] = x[:, k].copy()
    o.W_on = o.prox_on = 1
    o.iterk(iters, convthresh)
    return o


def all_certified(ph):
    """Every solve certified: the host loop's per-solve statistics and, when the
    device loop (phx_iterk) ran the iterations, its count of uncertified lanes."""
    return (all(s["not_optimal"] == 0 for s in ph.solve_stats)
            and getattr(ph, "iterk_stats", {}).get("not_optimal", 0) == 0)
