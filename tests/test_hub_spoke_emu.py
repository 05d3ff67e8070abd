"""The engine as the hub's and the Lagrangian spoke's opt object (SURVEY §8(b)
hub contract, §8(f) row 1), on CPU through the ABI emulation; GPU versions in
test_gpu_parity.py.

* hub: `spcomm.sync()` after Iter0 and after every iteration, `is_converged()`
  ending the loop (phbase.py:837-838, 953-957); the flat W and nonant buffers
  a PHHub sends (`send_ws` hub.py:590-598 via `_populate_W_cache` with 3
  trailing slots, `send_nonants` hub.py:562-577 via `_save_nonants`).
* Lagrangian spoke (cylinders/lagrangian_bounder.py:9-95): PHBase with
  PH_Prep(attach_prox=False) + _reenable_W, a solve with W = 0 (trivial bound),
  then W from the hub's flat buffer (W_from_flat_list) and Ebound with the
  serial-number extra sum term.
"""
import numpy as np

from helpers import ph_options, rel
from mpisppy_amd.examples import farmer
from mpisppy_amd.opt.ph import PH
from mpisppy_amd.phbase import PHBase
from oracle import models as om, ph as oph


class FakeHub:
    """spcomm stand-in with PHHub's sync/is_converged side of the contract."""

    def __init__(self, opt, stop_after=None):
        self.opt = opt
        self.stop_after = stop_after
        self.syncs = 0
        self.w_bufs = []
        self.nonant_bufs = []
        opt.spcomm = self

    def sync(self):
        self.syncs += 1
        opt = self.opt
        S, N = opt._S, opt.batch.nonant.N
        buf = np.zeros(S * N + 3)             # [W ... | outer, inner, write_id] (hub.py:281-285)
        opt._populate_W_cache(buf, padding=3)
        self.w_bufs.append(buf.copy())
        opt._save_nonants()
        flat = np.concatenate([s._mpisppy_data.nonant_cache for s in opt.local_scenarios.values()])
        self.nonant_bufs.append(flat)

    def is_converged(self):
        return self.stop_after is not None and self.syncs > self.stop_after


def check_hub(lib, device, S=12, iters=4):
    names = farmer.scenario_names_creator(S)
    ph = PH(ph_options(iters), names, farmer.scenario_creator, scenario_creator_kwargs={"num_scens": S},
            _native_lib=lib, _device=device)
    hub = FakeHub(ph)
    conv, Eobj, tb = ph.ph_main()
    assert not hasattr(ph, "iterk_stats")            # a hub needs the host loop
    assert hub.syncs == iters + 1                      # after Iter0 and after every iteration
    N = ph.batch.nonant.N
    assert np.array_equal(hub.w_bufs[-1][:S * N], ph.W_array().ravel())
    assert np.array_equal(hub.nonant_bufs[-1], ph.nonant_values().ravel())
    # the same trajectory as without a hub, bit for bit: the same host loop
    # (without a hub ph_main would run the device loop, whose fused reductions
    # sum in another fixed order -- agreement to 1e-9 there, tested in
    # test_native_loop_fused_matches_host_loop_gpu)
    ropts = ph_options(iters)
    ropts["iterk_solver_options"] = {"native_loop": 0}
    ref = PH(ropts, names, farmer.scenario_creator, scenario_creator_kwargs={"num_scens": S},
             _native_lib=lib, _device=device)
    rc, rE, rt = ref.ph_main()
    assert not hasattr(ref, "iterk_stats")
    assert np.array_equal(ref.W_array(), ph.W_array()) and rc == conv and rt == tb
    # is_converged ends iterk_loop right after the solve of that iteration
    ph2 = PH(ph_options(iters), names, farmer.scenario_creator, scenario_creator_kwargs={"num_scens": S},
             _native_lib=lib, _device=device)
    hub2 = FakeHub(ph2, stop_after=2)
    ph2.ph_main()
    assert ph2._PHIter == 2 and hub2.syncs == 3
    return ph, hub


def test_hub_contract_emu(emu):
    check_hub(emu, "cpu")


def check_lagrangian_spoke(lib, device, S=12, iters=4):
    names = farmer.scenario_names_creator(S)
    kw = {"num_scens": S}
    hub_opt = PH(ph_options(iters), names, farmer.scenario_creator, scenario_creator_kwargs=kw,
                 _native_lib=lib, _device=device)
    hub = FakeHub(hub_opt)
    hub_opt.ph_main()
    # the spoke's opt object (cfg_vanilla.lagrangian_spoke: opt_class = PHBase)
    opt = PHBase(ph_options(iters), names, farmer.scenario_creator, scenario_creator_kwargs=kw,
                 _native_lib=lib, _device=device)
    opt.PH_Prep(attach_prox=False)
    opt._reenable_W()
    opt.subproblem_creation(False)
    opt._create_solvers()
    assert opt.W_on == 1 and opt.prox_on == 0
    opt.solve_loop(solver_options=opt.current_solver_options, dtiming=False, gripe=True)
    trivial, extra = opt.Ebound(False, extra_sum_terms=[5])
    assert int(round(extra[0])) == 5
    assert rel(trivial, hub_opt.trivial_bound) < 1e-12
    # W from the hub's last send_ws buffer
    opt.W_from_flat_list(hub.w_bufs[-1][:-3])
    opt.solve_loop(solver_options=opt.current_solver_options, dtiming=False, gripe=True)
    bound = opt.Ebound(False)
    o = oph.OraclePH([om.farmer(n, num_scens=S) for n in names], rho=1.0)
    o.W = hub.w_bufs[-1][:-3].reshape(S, -1).copy()
    o.W_on, o.prox_on = 1, 0
    o.solve_loop()
    assert rel(bound, o.Ebound()) < 1e-9
    ef, _, st = oph.solve_ef([om.farmer(n, num_scens=S) for n in names])
    assert bound <= ef + 1e-6 * abs(ef)                # a valid outer (lower) bound
    assert bound >= trivial - 1e-6 * abs(trivial)      # and no worse than the trivial one here
    return bound, trivial, ef


def test_lagrangian_spoke_emu(emu):
    check_lagrangian_spoke(emu, "cpu")
