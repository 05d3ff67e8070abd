"""Hub and spokes as separate processes: a PHHub
running PH and a LagrangianOuterBound spoke, started by WheelSpinner over
torch.distributed (gloo) with the node-local shared-memory windows, on CPU
through the ABI emulation.

Checked against the reference's semantics (hub.py:370-598, spoke.py:60-208,
lagrangian_bounder.py:9-95, spin_the_wheel.py:34-159):
* wire format: the spoke reads `[W (S*N) | outer, inner, write_id]`, every
  bound it reports arrives with a write id, the kill signal is write id -1;
* every Lagrangian bound the spoke reported equals the oracle's Lagrangian bound
  (W on, prox off, exact LP/QP solves) for the hub's W of that write id;
* the hub's best outer bound is the best of those and the trivial bound, and
  lies below the EF optimum;
* 2 ranks per cylinder (world 4): scenarios sharded over the cylinder, write
  ids agreed across the cylinder's ranks, the same bounds as with 1 rank;
* three cylinders (hub + Lagrangian + x-bar inner bound, xhatxbar_bounder.py:31-114):
  the hub terminates on rel_gap (hub.py:125-161), each inner bound is the
  oracle's x-bar evaluation of the nonants it came from.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
S = 12
ITERS = 6


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out, gpu=False):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import mpisppy_amd  # noqa: F401
    from mpisppy_amd import _native
    from mpisppy_amd.comm import Comm
    from mpisppy_amd.cylinders import LagrangianOuterBound, PHHub
    from mpisppy_amd.examples import farmer
    from mpisppy_amd.opt.ph import PH
    from mpisppy_amd.phbase import PHBase
    from mpisppy_amd.spin_the_wheel import WheelSpinner
    from helpers import ph_options
    if gpu:     # the product library on cuda:0 (both cylinders share the one GPU)
        lib, device = _native.load(), "cuda:0"
    else:
        lib, device = _native.Lib(os.path.join(ROOT, "tests", "emu", "libphx_emu.so"), prefix="emu_phx_"), "cpu"
    names = farmer.scenario_names_creator(S)

    sent = []       # the hub's W per write id
    got = []        # the spoke's (write id, bound) per Lagrangian pass

    class RecordingHub(PHHub):
        def send_ws(self):
            super().send_ws()
            sent.append((int(self.w_send_buffer[-1]), self.w_send_buffer[:-3].copy()))

    class RecordingSpoke(LagrangianOuterBound):
        def lagrangian(self):
            b = super().lagrangian()
            got.append((int(self.get_serial_number()), b, self.localWs.copy()))
            return b

    okw = dict(options=ph_options(ITERS), all_scenario_names=names, scenario_creator=farmer.scenario_creator,
               scenario_creator_kwargs={"num_scens": S}, _native_lib=lib, _device=device)
    hub_dict = {"hub_class": RecordingHub, "hub_kwargs": {"options": {"display_progress": False}},
                "opt_class": PH, "opt_kwargs": dict(okw)}
    spoke_dict = {"spoke_class": RecordingSpoke, "opt_class": PHBase, "opt_kwargs": dict(okw)}
    wheel = WheelSpinner(hub_dict, [spoke_dict])
    wheel.spin(comm_world=Comm())
    sp = wheel.spcomm
    rec = {"strata_rank": wheel.strata_rank, "cylinder_rank": wheel.cylinder_rank,
           "local_names": list(sp.opt.local_scenario_names)}
    if wheel.strata_rank == 0:
        rec.update(best_outer=wheel.BestOuterBound, best_inner=wheel.BestInnerBound,
                   trivial=sp.opt.trivial_bound, sent=sent, write_ids=sp.local_write_ids.tolist(),
                   remote_ids=sp.remote_write_ids.tolist(), on_hub=wheel.on_hub(),
                   W=sp.opt.W_array())
    else:
        rec.update(got=got, final=sp.final_bound, remote_id=sp.remote_write_id,
                   local_id=sp.local_write_id, on_hub=wheel.on_hub())
    out[rank] = rec
    dist.barrier()
    dist.destroy_process_group()


def _run(world, gpu=False):
    mgr = mp.get_context("spawn").Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out, gpu), nprocs=world, join=True)
    return [out[r] for r in range(world)]


def _oracle_lagrangian(W_flat):
    from oracle import models as om, ph as oph
    names = ["scen%d" % i for i in range(S)]
    o = oph.OraclePH([om.farmer(n, num_scens=S) for n in names], rho=1.0)
    o.W = np.asarray(W_flat, dtype=np.float64).reshape(S, -1).copy()
    o.W_on, o.prox_on = 1, 0
    o.solve_loop()
    return o.Ebound()


def _check(res, ncyl, tol=1e-9):
    from oracle import models as om, ph as oph
    hubs = [r for r in res if r["strata_rank"] == 0]
    spokes = [r for r in res if r["strata_rank"] == 1]
    assert len(hubs) == ncyl and len(spokes) == ncyl
    assert all(h["on_hub"] for h in hubs) and not any(s["on_hub"] for s in spokes)
    # every cylinder covers all scenarios once (contiguous slices)
    for grp in (hubs, spokes):
        allnames = sorted(n for r in grp for n in r["local_names"])
        assert allnames == sorted("scen%d" % i for i in range(S))
    h0 = hubs[0]
    # sync after Iter0 and after every iteration: ITERS + 1 W sends, ids 1..ITERS+1
    ids = [i for i, _ in h0["sent"]]
    assert ids == list(range(1, ITERS + 2))
    assert h0["write_ids"] == [ITERS + 1]
    # full W vectors by write id (cylinder ranks hold slices: concatenate by rank)
    hub_ranks = sorted(hubs, key=lambda r: r["cylinder_rank"])
    W_by_id = {i: np.concatenate([dict(r["sent"])[i] for r in hub_ranks]) for i in ids}
    W_by_id[0] = np.zeros(S * 3)
    # the hub's final W is the last one sent (after the last iteration's solve)
    assert np.array_equal(np.concatenate([r["W"].ravel() for r in hub_ranks]), W_by_id[ITERS + 1])
    sp_ranks = sorted(spokes, key=lambda r: r["cylinder_rank"])
    g0 = sp_ranks[0]["got"]
    assert len(g0) >= 2
    # all spoke ranks ran the same passes with the same serial numbers and bounds
    for r in sp_ranks[1:]:
        assert [(i, b) for i, b, _ in r["got"]] == [(i, b) for i, b, _ in g0]
    # kill signal seen; the final pass ran on the kill buffer's zeros (reference quirk)
    assert all(r["remote_id"] == -1 for r in sp_ranks)
    bounds = []
    for k, (wid, b, _) in enumerate(g0):
        Wloc = np.concatenate([r["got"][k][2] for r in sp_ranks])
        if k == len(g0) - 1:               # finalize(): the buffer holds the kill signal's zeros
            assert not Wloc.any()
            continue
        assert np.array_equal(Wloc, W_by_id[wid]), wid
        ob = _oracle_lagrangian(W_by_id[wid])
        assert b == pytest.approx(ob, rel=tol, abs=1e-7), (wid, b, ob)
        bounds.append(b)
    # the spoke's first bound is the trivial bound (W = 0, serial number 0)
    assert g0[0][0] == 0 and g0[0][1] == pytest.approx(h0["trivial"], rel=1e-12)
    # the hub holds the best (largest: minimisation) bound it received, never worse than trivial
    ef, _, _ = oph.solve_ef([om.farmer("scen%d" % i, num_scens=S) for i in range(S)])
    assert h0["best_outer"] >= h0["trivial"] - 1e-9
    assert h0["best_outer"] <= ef + 1e-6 * abs(ef)
    # (the hub sees the values it happened to read: not every bound the spoke wrote;
    # it may read the final pass's, computed on the kill buffer's zeros -- a trivial
    # bound from a warm-started solve, equal to the trivial one to rounding)
    written = [b for _, b, _ in g0]
    # the final pass (kill buffer, W = 0, prox off) is the Iter0 problem again: its
    # bound is the trivial bound (the one unchecked value the hub may read)
    assert g0[-1][1] == pytest.approx(h0["trivial"], rel=1e-9)
    assert h0["best_outer"] in bounds + [g0[-1][1], h0["trivial"]]
    assert h0["best_outer"] <= max(written + [h0["trivial"]])
    assert h0["best_inner"] == float("inf")
    return [b for b in bounds]


def test_wheel_lagrangian_1x(emu):
    _check(_run(2), 1)


@pytest.mark.gpu
def test_wheel_lagrangian_gpu():
    """The same wheel (hub + Lagrangian spoke, two processes over gloo and the
    shared-memory windows) on the real kernels: both cylinders' contexts on
    cuda:0; every bound the spoke sent equals the oracle's for the W it read."""
    _check(_run(2, gpu=True), 1, tol=1e-8)


def test_wheel_lagrangian_2x(emu):
    """Two ranks per cylinder: sharded scenarios, write-id agreement."""
    _check(_run(4), 2)


def _worker3(rank, world, port, out):
    """hub + Lagrangian outer bound + x-bar inner bound, gap termination."""
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import mpisppy_amd  # noqa: F401
    from mpisppy_amd import _native
    from mpisppy_amd.comm import Comm
    from mpisppy_amd.cylinders import LagrangianOuterBound, PHHub, XhatXbarInnerBound
    from mpisppy_amd.examples import farmer
    from mpisppy_amd.opt.ph import PH
    from mpisppy_amd.phbase import PHBase
    from mpisppy_amd.spin_the_wheel import WheelSpinner
    from mpisppy_amd.utils.xhat_eval import Xhat_Eval
    from helpers import ph_options
    emu = _native.Lib(os.path.join(ROOT, "tests", "emu", "libphx_emu.so"), prefix="emu_phx_")
    names = farmer.scenario_names_creator(S)
    tried = []

    class RecordingXhat(XhatXbarInnerBound):
        def update_if_improving(self, b):
            tried.append((self.localnonants.copy(), b))
            return super().update_if_improving(b)

    okw = dict(options=ph_options(200), all_scenario_names=names, scenario_creator=farmer.scenario_creator,
               scenario_creator_kwargs={"num_scens": S}, _native_lib=emu, _device="cpu")
    xopts = dict(ph_options(200))
    xopts["xhat_xbar_options"] = {"xhat_solver_options": {}}
    hub_dict = {"hub_class": PHHub, "hub_kwargs": {"options": {"rel_gap": 0.01, "display_progress": False}},
                "opt_class": PH, "opt_kwargs": dict(okw)}
    spokes = [{"spoke_class": LagrangianOuterBound, "opt_class": PHBase, "opt_kwargs": dict(okw)},
              {"spoke_class": RecordingXhat, "opt_class": Xhat_Eval, "opt_kwargs": dict(okw, options=xopts)}]
    wheel = WheelSpinner(hub_dict, spokes)
    wheel.spin(comm_world=Comm())
    rec = {"strata_rank": wheel.strata_rank}
    if wheel.strata_rank == 0:
        rec.update(best_outer=wheel.BestOuterBound, best_inner=wheel.BestInnerBound,
                   iters=wheel.spcomm.opt._PHIter, last_ib_idx=wheel.spcomm.last_ib_idx)
    elif wheel.strata_rank == 2:
        rec.update(tried=tried, best=wheel.spcomm.best_inner_bound)
    out[rank] = rec
    dist.barrier()
    dist.destroy_process_group()


def test_wheel_three_cylinders_gap(emu):
    """PHHub + Lagrangian + x-bar spokes: the hub stops on rel_gap <= 1%; the
    inner bound is the oracle's evaluation of x-bar (nonants fixed, LPs
    re-solved) of the nonant vector it came from; outer <= EF <= inner."""
    from oracle import models as om, ph as oph
    mgr = mp.get_context("spawn").Manager()
    out = mgr.dict()
    mp.spawn(_worker3, args=(3, _free_port(), out), nprocs=3, join=True)
    res = [out[r] for r in range(3)]
    hub = [r for r in res if r["strata_rank"] == 0][0]
    xs = [r for r in res if r["strata_rank"] == 2][0]
    scens = [om.farmer("scen%d" % i, num_scens=S) for i in range(S)]
    ef, _, _ = oph.solve_ef(scens)
    assert hub["best_outer"] <= ef + 1e-6 * abs(ef) <= hub["best_inner"] + 2e-6 * abs(ef)
    gap = (hub["best_inner"] - hub["best_outer"]) / abs(hub["best_outer"])
    assert gap <= 0.01 and hub["iters"] < 200          # terminated on the gap, not the limit
    assert hub["last_ib_idx"] == 2
    # the spoke's evaluations, re-done by the oracle from the nonants it received
    feas = [(v, b) for v, b in xs["tried"] if b is not None]
    assert feas
    for v, b in feas[:3] + feas[-2:]:
        xb = v.reshape(S, -1).mean(axis=0)               # p = 1/S: x-bar of the ROOT node
        E, _, ok = oph.evaluate_xhat(scens, {"ROOT": xb})
        assert ok.all()
        assert b == pytest.approx(E, rel=1e-8, abs=1e-6)
    assert xs["best"] == pytest.approx(min(b for _, b in feas), rel=1e-12)


def test_window_seqlock_roundtrip():
    """The window's epoch protocol within one process: put / get round trip,
    write id slot, kill signal, and a torn epoch (odd sequence) is not read."""
    from mpisppy_amd.cylinders.spwindow import SPWindow
    a = SPWindow("t%d" % os.getpid(), 0, 0, [5, 3])
    b = SPWindow("t%d" % os.getpid(), 0, 1, [5, 3])
    try:
        v = np.arange(6, dtype=np.float64)
        v[-1] = 7
        a.put(v)
        out = np.zeros(6)
        b.get(0, out)
        assert np.array_equal(out, v)
        k = np.zeros(4)
        k[-1] = -1
        b.put(k)
        o2 = np.zeros(4)
        a.get(1, o2)
        assert o2[-1] == -1
        seq = SPWindow._seq(a._own)
        seq[0] += 1                       # a writer in the middle of an epoch
        with pytest.raises(RuntimeError):
            b.get(0, out, timeout=0.05)
        seq[0] += 1
        b.get(0, out)
    finally:
        out = o2 = None
        a.free()
        b.free()


def test_window_segments_unlinked_at_exit(tmp_path):
    """A process that creates a window and dies without free() (an exception in a
    spoke) leaves no segment behind: the atexit hook unlinks what it owns."""
    import subprocess
    import sys
    tag = "x%d" % os.getpid()
    code = ("import sys; sys.path.insert(0, %r)\n"
            "import mpisppy_amd\n"
            "from mpisppy_amd.cylinders.spwindow import SPWindow\n"
            "w = SPWindow(%r, 0, 0, [4])\n"
            "print(w._own.path)\n"
            "raise SystemExit(3)\n") % (os.path.dirname(os.path.dirname(os.path.abspath(__file__))), tag)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 3, r.stderr
    path = r.stdout.strip().splitlines()[-1]
    assert path.startswith("/dev/shm/phxw_" + tag)
    assert not os.path.exists(path)
