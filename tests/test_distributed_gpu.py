"""The N>1 device path on the GPU: several ranks, each its
own process and phx context on cuda:0, run the device-driven PH loop
(phx_iterk through the real libphx) with the per-iteration all-reduce issued
through the Python callback over gloo (two ranks on one device cannot share an
RCCL communicator; the callback enqueues on phx_iterk's stream, Comm.allreduce_
stages gloo's device tensors through the host).  Every multi-rank kernel path
runs on hardware here:

* the unfused loop's ``k_conv`` on the all-reduced per-rank convergence sums
  (phbase.py:330-343) and the stop it sets on every rank alike;
* the fused loop's one-launch iterations, whose staging buffer
  ``[x-bar sums | straggler count | conv sums]`` is all-reduced between launches
  (phbase.py:83-87, 341);
* straggler stops decided on the all-reduced straggler count (forced by starved
  lane solves): every rank stops, finishes its own leftovers, and resumes;
* the adopted Iter0's collective early exit: an infeasible scenario on rank 0
  only makes both ranks leave before any PH iteration (phbase.py:812-823).

Each multi-rank run is checked against the one-process run of the same
scenarios (conv_ranks = world size: the reference's per-rank normalisation,
sputils.py:803-810 slices).  Tolerances: the ranks' x-bar sums add in another
fixed order than one process's tiles (each rank's tiles, then the all-reduce),
so values agree to rounding, not bit for bit; the iteration counts are equal.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STRAG = {"as_rounds": 1, "ipm_max_it": 3, "rescue_rounds": 1}
CASES = {
    # name: (model, world, S or branching factors, iterations, convthresh, fused, solver options)
    "farmer-fused": ("farmer", 2, 2000, 60, 1.0, 1, None),
    "farmer-unfused": ("farmer", 2, 2000, 60, 1.0, 0, None),
    "farmer-strag-fused": ("farmer", 2, 2000, 8, 1e-10, 1, STRAG),
    "farmer-strag-unfused": ("farmer", 2, 2000, 8, 1e-10, 0, STRAG),
    "aircond3": ("aircond", 3, [5, 2, 2], 20, 1e-3, 1, None),
}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_case(case, lib, device, mpicomm=None, conv_ranks=None):
    from helpers import run_engine
    from mpisppy_amd.examples import aircond, farmer
    from mpisppy_amd.utils import sputils
    model, world, size, iters, thresh, fused, so = CASES[case]
    iterk = dict(so or {}, native_loop=1, iterk_fused=fused)
    opts = {"convthresh": thresh, "iter0_solver_options": dict(so or {}), "iterk_solver_options": iterk}
    if conv_ranks:
        opts["conv_ranks"] = conv_ranks
    if model == "farmer":
        ph, conv, Eobj, tb = run_engine(farmer.scenario_creator, farmer.scenario_names_creator(size),
                                        {"num_scens": size}, iters, lib=lib, device=device, mpicomm=mpicomm,
                                        options=opts)
    else:
        S = int(np.prod(size))
        ph, conv, Eobj, tb = run_engine(aircond.scenario_creator, ["scen%d" % i for i in range(S)],
                                        {"branching_factors": size, "start_seed": 0}, iters, lib=lib,
                                        device=device, mpicomm=mpicomm, options=opts,
                                        all_nodenames=sputils.create_nodenames_from_branching_factors(size))
    st = dict(ph.iterk_stats)
    st.pop("wall_s", None)
    st.pop("lane_warm_ms", None)
    return {"conv": conv, "Eobj": Eobj, "tb": tb, "W": ph.W_array(), "iters": ph._PHIter,
            "xbar": {k: v[0] for k, v in ph.xbar_by_node().items()}, "x": ph.nonant_values(), "stats": st,
            "n_local": len(ph.local_scenario_names)}


def _worker(rank, world, port, out, case):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import mpisppy_amd  # noqa: F401
    from mpisppy_amd import _native
    from mpisppy_amd.comm import Comm
    # (an exception ends this rank at once: mp.spawn then stops its peers)
    out[rank] = _run_case(case, _native.load(), "cuda:0", mpicomm=Comm())
    dist.barrier()
    dist.destroy_process_group()


def _rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.max(np.abs(a - b) / np.maximum(1.0, np.abs(b)))) if a.size else 0.0


@pytest.mark.gpu
@pytest.mark.timeout(600)
@pytest.mark.parametrize("case", list(CASES))
def test_ranks_match_one_gpu(gpu_lib, case):
    model, world, size, iters, thresh, fused, so = CASES[case]
    # (a spawned manager: the parent holds a GPU context, which a forked
    # child must not inherit)
    mgr = mp.get_context("spawn").Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out, case), nprocs=world, join=True)
    rs = [out[r] for r in range(world)]
    one = _run_case(case, gpu_lib, "cuda:0", conv_ranks=world)
    S = len(one["W"])
    assert [r["n_local"] for r in rs] == [int((g + 1) * S / world) - int(g * S / world) for g in range(world)]
    diffs = {}
    for g, r in enumerate(rs):
        st = r["stats"]
        # the multi-rank path ran on the device: fused where asked (two-stage, one
        # segment per rank), the same iteration count and stop as one process
        assert st["fused"] == bool(fused and model == "farmer"), st
        assert r["iters"] == one["iters"] and st["converged"] == one["stats"]["converged"], (st, one["stats"])
        assert st["not_optimal"] == 0
        if so:
            assert st["straggler_stops"] == rs[0]["stats"]["straggler_stops"] > 0, st
        diffs.setdefault("conv", []).append(_rel(r["conv"], one["conv"]))
        diffs.setdefault("Eobj", []).append(_rel(r["Eobj"], one["Eobj"]))
        assert r["tb"] == pytest.approx(one["tb"], rel=1e-12)
        for k, v in one["xbar"].items():
            diffs.setdefault("xbar", []).append(_rel(r["xbar"][k], v))
    if thresh < 1e-6:
        assert not one["stats"]["converged"]
    else:
        assert one["stats"]["converged"] and one["iters"] < iters
    W = np.vstack([r["W"] for r in rs])
    X = np.vstack([r["x"] for r in rs])
    diffs["W"] = [_rel(W, one["W"])]
    diffs["x"] = [_rel(X, one["x"])]
    print("[%s] max rel diffs vs one process: %s; iters %d, stats %s" % (
        case, {k: max(v) for k, v in diffs.items()}, one["iters"], rs[0]["stats"]))
    for k, v in diffs.items():
        assert max(v) < 1e-9, (k, diffs)


def _worker_infeasible(rank, world, port, out):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import mpisppy_amd  # noqa: F401
    from mpisppy_amd import _native
    from mpisppy_amd.comm import Comm
    from mpisppy_amd.opt.ph import PH
    from mpisppy_amd.examples import farmer
    from helpers import ph_options
    from test_engine_emu import infeasible_farmer_creator
    S = 30
    ph = PH(ph_options(20), farmer.scenario_names_creator(S), infeasible_farmer_creator,
            scenario_creator_kwargs={"num_scens": S}, _native_lib=_native.load(), _device="cuda:0",
            mpicomm=Comm())
    seen = []
    orig = ph._native.iterk

    def spy(ctx, so, a, res, stream):
        rc = orig(ctx, so, a, res, stream)
        seen.append((res._obj.iters, res._obj.solves, res._obj.adopted, res._obj.not_optimal))
        return rc
    ph._native.iterk = spy
    quit_ = False
    try:
        ph.ph_main()
    except SystemExit:
        quit_ = True
    out[rank] = (quit_, seen, len(ph.local_scenario_names))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_infeasible_deferred_iter0_two_ranks_gpu(gpu_lib):
    """The adopted Iter0 with an infeasible scenario on rank 0 only, on the
    GPU: the not-optimal count is all-reduced before any rank leaves phx_iterk,
    so both leave at iteration 0 and quit together."""
    # (a spawned manager: the parent holds a GPU context, which a forked
    # child must not inherit)
    mgr = mp.get_context("spawn").Manager()
    out = mgr.dict()
    mp.spawn(_worker_infeasible, args=(2, _free_port(), out), nprocs=2, join=True)
    for r in range(2):
        quit_, seen, nloc = out[r]
        assert quit_, r
        assert nloc == 15
        assert [s[:3] for s in seen] == [(0, 0, 1)], (r, seen)
    assert out[0][1][0][3] == 1 and out[1][1][0][3] == 0
