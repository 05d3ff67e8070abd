"""N>1 path on CPU: two gloo ranks (one 'GPU' each) give the same PH result as
one process; the fused allreduce replaces the per-node MPI reductions."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out, case):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import mpisppy_amd  # noqa: F401
    from mpisppy_amd import _native
    from mpisppy_amd.comm import Comm
    from helpers import run_engine
    from mpisppy_amd.examples import aircond, farmer
    from mpisppy_amd.utils import sputils
    emu = _native.Lib(os.path.join(ROOT, "tests", "emu", "libphx_emu.so"), prefix="emu_phx_")
    case, loop = case.split("-")
    bfs = [5, 2, 2] if case == "aircond3" else [3, 2, 2]
    # native: the device-driven loop (phx_iterk, all-reduce through the
    # callback); host: the Python loop (PHBase methods one by one)
    opts = {"iterk_solver_options": {"native_loop": 1 if loop == "native" else 0}}
    if case == "farmer":
        ph, conv, Eobj, tb = run_engine(farmer.scenario_creator, farmer.scenario_names_creator(9),
                                        {"num_scens": 9}, 4, lib=emu, device="cpu", mpicomm=Comm(), options=opts)
    else:
        S = int(np.prod(bfs))
        ph, conv, Eobj, tb = run_engine(aircond.scenario_creator, ["scen%d" % i for i in range(S)],
                                        {"branching_factors": bfs, "start_seed": 0}, 3, lib=emu, device="cpu",
                                        mpicomm=Comm(), options=opts,
                                        all_nodenames=sputils.create_nodenames_from_branching_factors(bfs))
    assert hasattr(ph, "iterk_stats") if loop == "native" else not hasattr(ph, "iterk_stats")
    out[rank] = (conv, Eobj, tb, ph.W_array(), {k: v[0] for k, v in ph.xbar_by_node().items()})
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("case", ["farmer-native", "farmer-host", "aircond-native", "aircond-host",
                                  "aircond3-native"])
def test_ranks_match_one(emu, case):
    """2 ranks; aircond3: 3 ranks over 20 scenarios of a 5x2x2 tree (uneven
    slices 6/7/7 that cut across second-stage nodes) through phx_iterk."""
    from helpers import run_engine
    from mpisppy_amd.examples import aircond, farmer
    from mpisppy_amd.utils import sputils
    mgr = mp.get_context("spawn").Manager()
    out = mgr.dict()
    world = 3 if case.startswith("aircond3") else 2
    mp.spawn(_worker, args=(world, _free_port(), out, case), nprocs=world, join=True)
    if case.startswith("farmer"):
        ph, conv, Eobj, tb = run_engine(farmer.scenario_creator, farmer.scenario_names_creator(9), {"num_scens": 9},
                                        4, lib=emu, device="cpu", options={"conv_ranks": 2})
    else:
        bfs = [5, 2, 2] if case.startswith("aircond3") else [3, 2, 2]
        S = int(np.prod(bfs))
        ph, conv, Eobj, tb = run_engine(aircond.scenario_creator, ["scen%d" % i for i in range(S)],
                                        {"branching_factors": bfs, "start_seed": 0}, 3, lib=emu, device="cpu",
                                        options={"conv_ranks": world},
                                        all_nodenames=sputils.create_nodenames_from_branching_factors(bfs))
    rs = [out[r] for r in range(world)]
    for r in rs:
        assert r[0] == pytest.approx(conv, rel=1e-12)
        assert r[1] == pytest.approx(Eobj, rel=1e-12)
        assert r[2] == pytest.approx(tb, rel=1e-12)
        for k, v in ph.xbar_by_node().items():
            assert np.allclose(r[4][k], v[0], rtol=1e-12, atol=1e-12)
    S = len(ph.W_array())
    assert [len(r[3]) for r in rs] == [int((g + 1) * S / world) - int(g * S / world) for g in range(world)]
    W = np.vstack([r[3] for r in rs])
    assert np.allclose(W, ph.W_array(), rtol=1e-10, atol=1e-9)


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
    emu = _native.Lib(os.path.join(ROOT, "tests", "emu", "libphx_emu.so"), prefix="emu_phx_")
    S = 30
    ph = PH(ph_options(20), farmer.scenario_names_creator(S), infeasible_farmer_creator,
            scenario_creator_kwargs={"num_scens": S}, _native_lib=emu, _device="cpu", mpicomm=Comm())
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


@pytest.mark.timeout(300)
def test_infeasible_deferred_iter0_two_ranks(emu):
    """the deferred Iter0 adopted by phx_iterk with an
    infeasible scenario on ONE rank: the stop decision is all-reduced, so both
    ranks leave the device loop before any PH iteration and quit together
    (phbase.py:812-823) instead of one rank waiting in iteration 1's all-reduce."""
    mgr = mp.get_context("spawn").Manager()
    out = mgr.dict()
    mp.spawn(_worker_infeasible, args=(2, _free_port(), out), nprocs=2, join=True)
    for r in range(2):
        quit_, seen, nloc = out[r]
        assert quit_, r
        assert nloc == 15
        assert [s[:3] for s in seen] == [(0, 0, 1)], (r, seen)
    assert out[0][1][0][3] == 1 and out[1][1][0][3] == 0      # the infeasible scenario is rank 0's
