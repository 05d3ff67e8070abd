"""WheelSpinner: top level of a hub-and-spoke run (spin_the_wheel.py:12-237).

One process per GPU (torchrun), ``n_proc`` a multiple of ``n_spokes + 1``:
global rank g is strata rank ``g % (n_spokes + 1)`` (0 = hub) of strata group
``g // (n_spokes + 1)``, and cylinder rank ``g // (n_spokes + 1)`` of its
cylinder (the reference's ``_make_comms``).  Each cylinder's opt object gets
its cylinder communicator as ``mpicomm`` and shards the scenarios over it.
"""
from .comm import Comm, init_from_env
from .spbase import _global_toc as global_toc


class WheelSpinner:
    def __init__(self, hub_dict, list_of_spoke_dict):
        self.hub_dict = hub_dict
        self.list_of_spoke_dict = list_of_spoke_dict
        self._ran = False

    def spin(self, comm_world=None):
        return self.run(comm_world=comm_world)

    def run(self, comm_world=None):
        if self._ran:
            raise RuntimeError("WheelSpinner can only be run once")
        hub_dict = self.hub_dict
        list_of_spoke_dict = self.list_of_spoke_dict
        if "hub_class" not in hub_dict:
            raise RuntimeError("The hub_dict must contain a 'hub_class' key specifying the hub class to use")
        if "opt_class" not in hub_dict:
            raise RuntimeError("The hub_dict must contain an 'opt_class' key specifying "
                               "the SPBase class to use (e.g. PHBase, etc.)")
        hub_dict.setdefault("hub_kwargs", dict())
        hub_dict.setdefault("opt_kwargs", dict())
        for spoke_dict in list_of_spoke_dict:
            if "spoke_class" not in spoke_dict:
                raise RuntimeError("Each spoke_dict must contain a 'spoke_class' key "
                                   "specifying the spoke class to use")
            if "opt_class" not in spoke_dict:
                raise RuntimeError("Each spoke_dict must contain an 'opt_class' key "
                                   "specifying the SPBase class to use (e.g. PHBase, etc.)")
            spoke_dict.setdefault("spoke_kwargs", dict())
            spoke_dict.setdefault("opt_kwargs", dict())

        fullcomm = comm_world if comm_world is not None else init_from_env()
        n_spokes = len(list_of_spoke_dict)
        strata_comm, cylinder_comm = _make_comms(n_spokes, fullcomm=fullcomm)
        strata_rank = strata_comm.Get_rank()
        cylinder_rank = cylinder_comm.Get_rank()
        global_rank = fullcomm.Get_rank()

        if strata_rank == 0:
            sp_class, sp_kwargs = hub_dict["hub_class"], hub_dict["hub_kwargs"]
            opt_class, opt_kwargs = hub_dict["opt_class"], hub_dict["opt_kwargs"]
            opt_dict = hub_dict
        else:
            spoke_dict = list_of_spoke_dict[strata_rank - 1]
            sp_class, sp_kwargs = spoke_dict["spoke_class"], spoke_dict["spoke_kwargs"]
            opt_class, opt_kwargs = spoke_dict["opt_class"], spoke_dict["opt_kwargs"]
            opt_dict = spoke_dict

        opt_kwargs["mpicomm"] = cylinder_comm
        opt = opt_class(**opt_kwargs)
        if strata_rank == 0:
            spcomm = sp_class(opt, fullcomm, strata_comm, cylinder_comm, list_of_spoke_dict, **sp_kwargs)
        else:
            spcomm = sp_class(opt, fullcomm, strata_comm, cylinder_comm, **sp_kwargs)

        spcomm.make_windows()
        if strata_rank == 0:
            spcomm.setup_hub()
        global_toc("Starting spcomm.main()", global_rank == 0)
        spcomm.main()
        if strata_rank == 0:
            spcomm.send_terminate()
        spcomm.finalize()
        cylinder_comm.Barrier()
        global_toc(f"Hub algorithm {opt_class.__name__} complete, waiting for spoke finalization",
                   global_rank == 0)
        fullcomm.Barrier()
        # the hub catches the spokes' last values
        spcomm.hub_finalize()
        fullcomm.Barrier()
        spcomm.free_windows()

        self.spcomm = spcomm
        self.opt_dict = opt_dict
        self.global_rank = global_rank
        self.strata_rank = strata_rank
        self.cylinder_rank = cylinder_rank
        if strata_rank == 0:
            self.BestInnerBound = spcomm.BestInnerBound
            self.BestOuterBound = spcomm.BestOuterBound
        else:
            self.BestInnerBound = None
            self.BestOuterBound = None
        self._ran = True

    def on_hub(self):
        if not self._ran:
            raise RuntimeError("Need to call WheelSpinner.run() before finding out.")
        return "hub_class" in self.opt_dict

    def local_nonant_cache(self):
        """Nonant values per local tree node (spin_the_wheel.py:192-204)."""
        if not self._ran:
            raise RuntimeError("Need to call WheelSpinner.run() before querying solutions.")
        opt = self.spcomm.opt
        vals = opt.nonant_values()
        local_xhats = dict()
        for sname, view in opt.local_scenarios.items():
            per_node = dict()
            for j, (ndn, i) in enumerate(view._keys()):
                per_node.setdefault(ndn, []).append(float(vals[view._s, j]))
            for ndn, v in per_node.items():
                local_xhats.setdefault(ndn, v)
        return local_xhats


def _make_comms(n_spokes, fullcomm=None):
    """spin_the_wheel.py:219-237."""
    nsp1 = n_spokes + 1
    if fullcomm is None:
        fullcomm = Comm()
    n_proc = fullcomm.Get_size()
    if n_proc % nsp1 != 0:
        raise RuntimeError(f"Need a multiple of {nsp1} processes (got {n_proc})")
    global_rank = fullcomm.Get_rank()
    strata_comm = fullcomm.Split(color=global_rank // nsp1, key=global_rank)
    cylinder_comm = fullcomm.Split(color=global_rank % nsp1, key=global_rank)
    return strata_comm, cylinder_comm
