"""SPBase — scenario distribution and the device-resident scenario batch.

Mirrors ``mpisppy.spbase.SPBase`` (``mpisppy/spbase.py:44-120``): same
constructor, same contiguous rank slicing (``_calculate_scenario_ranks``
184-216 / ``sputils._ScenTree`` 774-840), same default uniform probability
(``_look_and_leap`` 505-522), same ``prob_coeff = p_s / uncond_prob(node)``
(``_compute_unconditional_node_probabilities`` 378-391), same nonant index
order (``_attach_nonant_indices`` 293-302) and the same errors
(``RuntimeError("More ranks than scenarios")``, ``ValueError`` for missing
options).

Instead of one Pyomo model per scenario, the local scenarios live as ONE
batch on the GPU (scenario-minor tensors, see ``batch.py``) behind a native
context (``libphx``).  Per-tree-node MPI communicators
(``_create_communicators`` 333-375) are replaced by a segment map: scenarios of
a node are contiguous, node sums are local segmented reductions followed by a
single fused allreduce.
"""
import ctypes
import math
import os
import time
import weakref

import numpy as np
import torch

from . import _native
from . import batch as batchmod
from .comm import Comm, init_from_env
from .utils import sputils


def _global_toc(msg, cond=True):
    if cond:
        print("[%8.2f] %s" % (time.perf_counter() - _T0, msg), flush=True)


_T0 = time.perf_counter()


class SPBase:
    def __init__(self, options, all_scenario_names, scenario_creator, scenario_denouement=None,
                 all_nodenames=None, mpicomm=None, scenario_creator_kwargs=None,
                 variable_probability=None, E1_tolerance=1e-5, _native_lib=None, _device=None):
        self.start_time = time.perf_counter()
        self.options = options
        self.all_scenario_names = list(all_scenario_names)
        self.scenario_creator = scenario_creator
        self.scenario_denouement = scenario_denouement
        self.comms = dict()
        self.local_scenarios = dict()
        self.local_scenario_names = list()
        self.E1_tolerance = E1_tolerance
        self.names_in_bundles = None
        self.scenarios_constructed = False
        if all_nodenames is None:
            self.all_nodenames = ["ROOT"]
        elif "ROOT" in all_nodenames:
            self.all_nodenames = list(all_nodenames)
            self._check_nodenames()
        else:
            raise RuntimeError("'ROOT' must be in the list of node names")
        # per-variable probabilities (spbase.py:394-434): needs the per-scenario models
        self.variable_probability = variable_probability
        if variable_probability is not None:
            self.options["per_scenario_models"] = True
        self.multistage = len(self.all_nodenames) > 1
        if mpicomm is None:
            # under torchrun (WORLD_SIZE > 1) join the process group: RCCL for GPU
            # tensors, gloo when the caller runs the engine on CPU tensors
            dev_type = "cuda" if _device is None else torch.device(_device).type
            mpicomm = init_from_env(dev_type)
        self.mpicomm = mpicomm
        self.cylinder_rank = self.mpicomm.Get_rank()
        self.n_proc = self.mpicomm.Get_size()
        self.global_rank = self.cylinder_rank
        if options.get("toc", True) and self.cylinder_rank == 0 and options.get("verbose", False):
            _global_toc("Initializing SPBase")
        if self.n_proc > len(self.all_scenario_names):
            raise RuntimeError("More ranks than scenarios")
        self._calculate_scenario_ranks()
        # EF bundles (spbase.py:219-253): bundles_per_rank slices of each rank's scenarios
        self.bundling = int(self.options.get("bundles_per_rank", 0) or 0) > 0
        if self.bundling and self.n_proc * int(self.options["bundles_per_rank"]) > len(self.all_scenario_names):
            raise RuntimeError("Not enough scenarios to satisfy the bundles_per_rank requirement")
        self._native = _native_lib if _native_lib is not None else _native.load()
        if _device is None:
            if not torch.cuda.is_available():
                raise _native.NativeError("no GPU visible: the batched PH engine runs on MI355X only "
                                          "(there is no CPU fallback)")
            _device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(_device)
        self._create_scenarios(scenario_creator_kwargs)
        self._look_and_leap()
        self._set_sense()
        self._compute_unconditional_node_probabilities()
        self._attach_nonant_indices()
        self._use_variable_probability_setter()
        self._create_communicators()
        self._upload_batch()
        self._bundles = None
        self._prox_lin = None          # linearised prox terms (prox_approx.ProxLinSolver), PHBase sets it
        if self.bundling:
            self._setup_bundles()
        self._spcomm = None
        self.tree_solution_available = False
        self.first_stage_solution_available = False

    def _setup_bundles(self):
        """The bundles of this rank (names_in_bundles as the reference holds it:
        {rank: {bundle: [scenario names]}}) and their device solver."""
        from .bundles import BundleSolver, assign_bundles
        B = int(self.options["bundles_per_rank"])
        groups = assign_bundles(len(self.local_scenario_names), B)
        self.names_in_bundles = {self.cylinder_rank: {g: [self.local_scenario_names[k] for k in grp]
                                                      for g, grp in enumerate(groups)}}
        self._bundles = BundleSolver(self, groups)

    # ------------------------------------------------------------ tree/ranks
    def _check_nodenames(self):
        names = set(self.all_nodenames)
        for ndn in self.all_nodenames:
            if ndn != "ROOT" and sputils.parent_ndn(ndn) not in names:
                raise RuntimeError("all_nodenames is inconsistent:The node %s, parent of %s, is missing."
                                   % (sputils.parent_ndn(ndn), ndn))

    def _calculate_scenario_ranks(self):
        S = len(self.all_scenario_names)
        self._rank_bounds = sputils.rank_bounds(S, self.n_proc)
        self._rank_slices = [list(range(a, b)) for a, b in self._rank_bounds]
        lo, hi = self._rank_bounds[self.cylinder_rank]
        self._local_lo, self._local_hi = lo, hi
        self.local_scenario_names = self.all_scenario_names[lo:hi]
        leaf = sputils.find_leaves(self.all_nodenames)
        self.nonleaves = [nd for nd in self.all_nodenames if not leaf.get(nd, False)]

    def _create_scenarios(self, scenario_creator_kwargs):
        if self.scenarios_constructed:
            raise RuntimeError("Scenarios already constructed.")
        kw = dict(scenario_creator_kwargs or {})
        t0 = time.time()
        bc = getattr(self.scenario_creator, "batch_creator", None)
        self._models = None
        if bc is not None and not self.options.get("per_scenario_models", False):
            data = bc(self.local_scenario_names, **kw)
        else:
            models = [self.scenario_creator(nm, **kw) for nm in self.local_scenario_names]
            self._models = dict(zip(self.local_scenario_names, models))
            data = batchmod.from_models(self.local_scenario_names, models)
        self.batch = data
        self._instance_creation_time = time.time() - t0
        if self.options.get("display_timing", False):
            allt = self.mpicomm.gather(self._instance_creation_time)
            if self.cylinder_rank == 0:
                print("Scenario instance creation times: total per rank max=%.2f" % max(allt))
        self.scenarios_constructed = True

    def _look_and_leap(self):
        S = len(self.all_scenario_names)
        probs = np.empty(self.batch.S)
        warned = False
        for k, p in enumerate(list(self.batch.prob)):
            if p is None or p == "uniform" or (isinstance(p, float) and math.isnan(p)):
                if not warned and self.cylinder_rank == 0 and p is None:
                    print("Did not find _mpisppy_probability, assuming uniform probability %s" % (1.0 / S))
                    warned = True
                probs[k] = 1.0 / S
            else:
                probs[k] = float(p)
        # (read-only from here: the cached sum below stays valid)
        probs.flags.writeable = False
        self.batch.prob = probs
        # the local probability sum, once (host data fixed from here): Iter0's
        # E1 check reads it instead of summing S values in the timed Iter0
        # (phbase.py _can_defer_iter0; keyed by the array object it summed --
        # held here, so a replacement array can never pass for it)
        self._prob_local_sum = (probs, float(np.sum(probs)))

    def _set_sense(self):
        senses = self.mpicomm.allgather_object(self.batch.sense)
        if any(v != senses[0] for v in senses):
            raise RuntimeError("All scenario models must have the same model sense (minimize or maximize)")
        self.is_minimizing = self.batch.sense == 1

    def _compute_unconditional_node_probabilities(self):
        nn = self.batch.nonant
        S = self.batch.S
        T = nn.nstages
        uncond = [np.ones(S)]
        for t in range(1, T):
            uncond.append(uncond[t - 1] * nn.cond_prob[t])
        self._uncond = uncond
        pc = np.empty((nn.N, S))
        for j in range(nn.N):
            t = nn.slot_stage[j] - 1
            pc[j] = self.batch.prob / uncond[t]
        self._prob_coeff = pc

    def _use_variable_probability_setter(self, verbose=False):
        """Per-variable probabilities from ``variable_probability(model, **kw)``
        -> [(id(var), prob)] (spbase.py:394-434): they replace the nonant slot's
        prob_coeff for that scenario; a zero probability masks the slot's W
        (prob0_mask, phbase.py:314-318).  Checked to sum to one per node and
        variable unless options['do_not_check_variable_probabilities']."""
        self._prob0_mask = None
        self._has_variable_probability = self.variable_probability is not None
        if self.variable_probability is None:
            return
        kw = self.options.get("variable_probability_kwargs", dict())
        nn = self.batch.nonant
        col_to_slot = {int(c): j for j, c in enumerate(nn.slot_col)}
        mask = np.ones((nn.N, self.batch.S))
        didit = 0
        for s, sname in enumerate(self.local_scenario_names):
            mdl = self._models[sname]
            byid = {id(v): v for v in mdl._vars}
            for vid, prob in self.variable_probability(mdl, **kw):
                v = byid.get(vid)
                if v is None or int(v.index) not in col_to_slot:
                    raise KeyError(vid)       # the reference's varid_to_nonant_index lookup
                j = col_to_slot[int(v.index)]
                self._prob_coeff[j, s] = float(prob)
                if prob == 0:
                    mask[j, s] = 0.0
                didit += 1
        self._prob0_mask = mask
        if verbose and self.cylinder_rank == 0:
            print("variable_probability set", didit)
        if not self.options.get("do_not_check_variable_probabilities", False):
            self._check_variable_probabilities_sum(verbose)

    def _check_variable_probabilities_sum(self, verbose=False):
        """Per node and nonant: sum of the slot probabilities over scenarios == 1
        (spbase.py:455-503)."""
        nn = self.batch.nonant
        loc = {}
        for s in range(self.batch.S):
            for j in range(nn.N):
                key = (nn.node_of(nn.slot_stage[j] - 1, s), j)
                loc[key] = loc.get(key, 0.0) + float(self._prob_coeff[j, s])
        tot = {}
        for d in self.mpicomm.allgather_object(loc):
            for k, v in d.items():
                tot[k] = tot.get(k, 0.0) + v
        bad = {}
        for (ndn, j), v in sorted(tot.items()):
            if not np.isclose(v, 1.0, atol=self.E1_tolerance):
                bad.setdefault(ndn, []).append((nn.var_names[j], v))
        for ndn, lst in bad.items():
            raise RuntimeError(f"Node {ndn}, variables {[a for a, _ in lst]} have respective"
                               f" conditional probability sum {[b for _, b in lst]}"
                               " which are not 1")

    def is_zero_prob(self, scenario_model, var):
        """spbase.py:436-452."""
        if self.variable_probability is None:
            return False
        names = [k for k, m in (self._models or {}).items() if m is scenario_model]
        if not names:
            view = getattr(scenario_model, "_s", None)          # a ScenarioView
            if view is None:
                return False
            s = view
        else:
            s = self.local_scenario_names.index(names[0])
        j = list(self.batch.nonant.slot_col).index(var.index)
        return float(self._prob_coeff[j, s]) == 0.0

    def _attach_nonant_indices(self):
        nn = self.batch.nonant
        # (ndn, i) keys of the first local scenario, node-list order
        self.nonant_length = nn.N
        self._slot_keys_cache = {}

    def slot_keys(self, s):
        """[(ndn, i)] of local scenario s in slot order (``nonant_indices`` keys)."""
        nn = self.batch.nonant
        return [(nn.node_of(nn.slot_stage[j] - 1, s), int(nn.slot_local[j])) for j in range(nn.N)]

    def _create_communicators(self):
        """Node -> contiguous scenario segments; global (node, slot) offsets."""
        nn = self.batch.nonant
        S = self.batch.S
        T = nn.nstages
        nlen = [nn.nlen(t) for t in range(T)]
        # non-leaf nodes in all_nodenames order, stage by name depth
        if self.multistage:
            nodes = [nd for nd in self.nonleaves]
        else:
            nodes = ["ROOT"]
        stage_of = {nd: nd.count("_") + 1 for nd in nodes}
        for nd in nodes:
            if stage_of[nd] > T:
                raise RuntimeError("Tree node %s has no nonant slots (stage %d > %d)" % (nd, stage_of[nd], T))
        self._node_names = nodes
        self._node_index = {nd: v for v, nd in enumerate(nodes)}
        node_off = np.zeros(len(nodes), dtype=np.int64)
        off = 0
        for v, nd in enumerate(nodes):
            node_off[v] = off
            off += nlen[stage_of[nd] - 1]
        self._node_off = node_off
        self._node_nlen = np.array([nlen[stage_of[nd] - 1] for nd in nodes], dtype=np.int64)
        self.NNS = off
        # per stage: node id of each local scenario; contiguity check
        node_id = np.zeros((T, S), dtype=np.int64)
        for t in range(T):
            if nn.node_names[t] is None:
                node_id[t] = self._node_index["ROOT"]
            else:
                try:
                    node_id[t] = [self._node_index[x] for x in nn.node_names[t]]
                except KeyError as e:
                    raise RuntimeError("Tree node %s not in all_nodenames list" % e)
        self._local_node_id = node_id
        # xbar index per (slot, scenario)
        xbar_idx = np.empty((nn.N, S), dtype=np.int64)
        for j in range(nn.N):
            t = nn.slot_stage[j] - 1
            xbar_idx[j] = node_off[node_id[t]] + nn.slot_local[j]
        self._xbar_idx = xbar_idx
        # tiles for the segmented xbar reduction
        CH = int(self.options.get("xbar_tile", 256))
        slot_lo = [int(np.argmax(nn.slot_stage == t + 1)) for t in range(T)]
        tiles = []   # (node v, s0, s1, slot0, nlen)
        for t in range(T):
            ids = node_id[t]
            if S == 0:
                continue
            starts = np.concatenate([[0], np.nonzero(np.diff(ids))[0] + 1, [S]])
            seen = set()
            for a, b in zip(starts[:-1], starts[1:]):
                v = int(ids[a])
                if v in seen:
                    raise RuntimeError("scenarios of tree node %s are not contiguous" % nodes[v])
                seen.add(v)
                for s0 in range(int(a), int(b), CH):
                    tiles.append((v, s0, min(int(b), s0 + CH), slot_lo[t], nlen[t]))
        tiles.sort(key=lambda x: (x[0], x[1]))
        self._tiles = tiles
        # the reference's per-node comms: here a name->segment map
        for nd in nodes:
            self.comms[nd] = self.mpicomm
        # emulated reference ranks for convergence_diff (phbase.py:330-343)
        R = int(self.options.get("conv_ranks", self.n_proc))
        Sg = len(self.all_scenario_names)
        vb = sputils.rank_bounds(Sg, R)
        lo, hi = self._local_lo, self._local_hi
        self._conv_R = R
        self._conv_counts = np.array([(b - a) * nn.N for a, b in vb], dtype=np.float64)
        # (each emulated rank's scenarios clipped to this rank's slice, in local
        # indices; an emulated rank outside the slice is an empty segment inside it)
        def clip(a, b):
            a = min(max(a, lo), hi)
            return a - lo, max(min(b, hi), a) - lo
        self._conv_seg = [clip(a, b) for a, b in vb]

    # ------------------------------------------------------------ device
    def _t(self, a, dtype):
        a = np.ascontiguousarray(a)
        if not a.flags.writeable:          # (the read-only probabilities: torch wants a writable buffer)
            a = a.copy()
        return torch.as_tensor(a, dtype=dtype).to(self.device)

    def _upload_batch(self):
        b = self.batch
        b.compress()
        f64, i32 = torch.float64, torch.int32
        S, n, m, N = b.S, b.n, b.m, b.nonant.N
        self._S = S
        # internal problems are minimisations; max problems are negated (see spopt)
        sgn = 1.0 if self.is_minimizing else -1.0
        c = b.c * sgn
        # the objective constant (c0, e.g. a Pyomo expression's constant term) is not
        # part of the device problem: it is added where objectives are read out
        # (_host obj/outer, Eobjective, Ebound, objs_dict), in the internal min sense
        self._c0_int = np.asarray(b.c0, dtype=np.float64) * sgn
        self._pc0 = math.fsum(float(p) * float(v) for p, v in zip(b.prob, self._c0_int))
        self._pc0_sum = float(self.mpicomm.allreduce_np([self._pc0])[0])   # over ranks (Ebound / Eobjective)
        d = {}
        d["rowptr"] = self._t(b.rowptr, i32)
        d["colidx"] = self._t(b.colidx, i32)
        d["kvar"] = self._t(b.kvar, i32)
        d["Aconst"] = self._t(b.Aconst, f64)
        d["Avar"] = self._t(b.Avar.ravel() if b.nvar else np.zeros(1), f64)
        d["c"] = self._t(b.minor(c, b.c_vary), f64)
        d["lb"] = self._t(b.minor(b.lb, b.bnd_vary), f64)
        d["ub"] = self._t(b.minor(b.ub, b.bnd_vary), f64)
        d["bl"] = self._t(b.minor(b.bl, b.rhs_vary) if m else np.zeros(1), f64)
        d["bu"] = self._t(b.minor(b.bu, b.rhs_vary) if m else np.zeros(1), f64)
        d["slot_col"] = self._t(b.nonant.slot_col if N else np.zeros(1, np.int32), i32)
        self._dev = d
        lib = self._native
        ctx = ctypes_void()
        lib.check(None, lib.create(int(self.device.index or 0), ctypes.byref(ctx)), "create")
        self._ctx = ctx.value
        weakref.finalize(self, lib.destroy, self._ctx)
        desc = _native.ProblemDesc()
        desc.S, desc.n, desc.m, desc.nnz, desc.N, desc.nvar = S, n, m, b.nnz, N, b.nvar
        for k in ["rowptr", "colidx", "kvar", "Aconst", "Avar", "c", "lb", "ub", "bl", "bu", "slot_col"]:
            setattr(desc, k, d[k].data_ptr())
        desc.c_vary, desc.bnd_vary, desc.rhs_vary = int(b.c_vary), int(b.bnd_vary), int(b.rhs_vary)
        # lane-solver tuning compiled with the problem (solver options
        # lane_multi_theta / lane_multi_rounds; iterk's over iter0's)
        so = dict(self.options.get("iter0_solver_options") or {})
        so.update(self.options.get("iterk_solver_options") or {})
        desc.lane_multi_theta = float(so.get("lane_multi_theta", 0.0) or 0.0)
        desc.lane_multi_rounds = int(so.get("lane_multi_rounds", 0) or 0)
        lib.check(self._ctx, lib.set_problem(self._ctx, desc), "set_problem")
        self._desc = desc
        # PH state
        self._x = torch.zeros(n * S, dtype=f64, device=self.device)
        self._x_touched = False          # x still all zeros (SPOpt._save_original_nonants)
        self._y = torch.zeros(max(m, 1) * S, dtype=f64, device=self.device)
        self._obj = torch.zeros(S, dtype=f64, device=self.device)
        self._iter0_obj_dev = torch.zeros(S, dtype=f64, device=self.device)   # Iter0's optima (PHBase)
        self._iter0_status_dev = torch.zeros(S, dtype=i32, device=self.device)  # ... and statuses
        # nonant slot -> column, and the original-nonant copy (SPOpt._save_original_nonants)
        self._slot_cols_dev = torch.as_tensor(self.batch.nonant.slot_col.astype(np.int64), device=self.device)
        self._orig_nonants_dev = torch.zeros((self.batch.nonant.N, S), dtype=f64, device=self.device)
        # the batched solve is exact (KKT-certified), so each scenario's outer
        # bound is its optimal objective (spopt.py:201-206): one buffer
        self._outer = self._obj
        self._status = torch.zeros(S, dtype=i32, device=self.device)
        self._iters = torch.zeros(S, dtype=i32, device=self.device)
        self._prob = self._t(b.prob, f64)
        self._pc = self._t(self._prob_coeff.ravel(), f64)
        self._prob0_mask_t = (None if getattr(self, "_prob0_mask", None) is None
                              else self._t(self._prob0_mask.ravel(), f64))
        self._xbar_idx_t = self._t(self._xbar_idx.ravel(), i32)
        # [sum p x | sum p x^2] per (node, slot), all-reduced in place; xbar and
        # xsqbar are views of it (no copies per iteration)
        self._node_buf = torch.zeros(max(2 * self.NNS, 2), dtype=f64, device=self.device)
        NNS1 = max(self.NNS, 1)
        self._xbar_node = self._node_buf[:NNS1]
        self._xsqbar_node = self._node_buf[NNS1:2 * NNS1]
        # phx_iterk: this iteration's sums (+ the straggler count, + the
        # per-emulated-rank conv sums in the fused mode), all-reduced before
        # they are published into _node_buf
        self._node_stage = torch.zeros(2 * NNS1 + 1 + self._conv_R, dtype=f64, device=self.device)
        self._dsum = torch.zeros(S, dtype=f64, device=self.device)
        # per-emulated-rank |x - xbar| sums + one slot for the straggler count of
        # a deferred solve (all-reduced together, phbase.convergence_diff)
        self._seg_sums = torch.zeros(self._conv_R + 1, dtype=f64, device=self.device)
        self._expect_buf = torch.zeros(3, dtype=f64, device=self.device)
        # tree descriptor
        tiles = self._tiles
        out = []
        o = 0
        for t in tiles:
            out.append(o)
            o += 2 * t[4]
        node_ids = sorted(set(t[0] for t in tiles))
        ptr = [0]
        for v in node_ids:
            ptr.append(ptr[-1] + sum(1 for t in tiles if t[0] == v))
        td = {}
        td["s0"] = self._t(np.array([t[1] for t in tiles] or [0], np.int32), i32)
        td["s1"] = self._t(np.array([t[2] for t in tiles] or [0], np.int32), i32)
        td["slot"] = self._t(np.array([t[3] for t in tiles] or [0], np.int32), i32)
        td["nlen"] = self._t(np.array([t[4] for t in tiles] or [0], np.int32), i32)
        td["out"] = self._t(np.array(out or [0], np.int32), i32)
        td["ptr"] = self._t(np.array(ptr, np.int32), i32)
        td["noff"] = self._t(np.array([self._node_off[v] for v in node_ids] or [0], np.int32), i32)
        td["nl"] = self._t(np.array([self._node_nlen[v] for v in node_ids] or [0], np.int32), i32)
        self._partial = torch.zeros(max(o, 1), dtype=f64, device=self.device)
        tree = _native.TreeDesc()
        tree.ntiles = len(tiles)
        tree.tile_s0, tree.tile_s1 = td["s0"].data_ptr(), td["s1"].data_ptr()
        tree.tile_slot, tree.tile_nlen, tree.tile_out = td["slot"].data_ptr(), td["nlen"].data_ptr(), td["out"].data_ptr()
        tree.nnodes = len(node_ids)
        tree.node_tile_ptr, tree.node_off, tree.node_nlen = td["ptr"].data_ptr(), td["noff"].data_ptr(), td["nl"].data_ptr()
        tree.NNS = self.NNS
        tree.npart = o
        tree.nnodes_cover = int(sum(int(self._node_nlen[v]) for v in node_ids))
        tree.node_key = self._xbar_idx_t.data_ptr()
        self._tree = tree
        self._tree_t = td
        segs = self._conv_seg
        self._seg_s0 = (_native.c_int32 * len(segs))(*[a for a, _ in segs])
        self._seg_s1 = (_native.c_int32 * len(segs))(*[b for _, b in segs])
        self._host_epoch = 0
        self._host_cache = {}
        # the stream handle and the small pinned buffer, looked up / allocated now
        # rather than inside the first timed PH step
        self._stream()
        if self.device.type == "cuda":
            self._pinned_small()
        # Iter0's expectation sums as phx_iterk leaves them (pinned on GPUs)
        self._iter0_exp_host = torch.zeros(3, dtype=f64, pin_memory=self.device.type == "cuda")

    def _stream(self):
        """The stream every native call is ordered on: the device's current
        stream when the object was built (its handle cached: looking it up
        costs more than most kernel launches)."""
        h = getattr(self, "_stream_h", None)
        if h is None:
            h = self._stream_h = (torch.cuda.current_stream(self.device).cuda_stream
                                  if self.device.type == "cuda" else 0)
        return h or None

    def _check_stream(self):
        """The torch ops between native calls (small reads, events, masks) run on
        the device's current stream; they are ordered after the native kernels
        only while that is still the stream cached by ``_stream``.  Checked once
        per entry point (Iter0, iterk_loop, small reads), not per call: running
        a built object inside another ``torch.cuda.stream(...)`` context raises
        instead of reading stale values."""
        if self.device.type != "cuda":
            return
        self._stream()
        # (the raw handle: torch.cuda.current_stream builds a Stream object, ~7 us)
        cur = torch._C._cuda_getCurrentRawStream(self.device.index or 0)
        if cur != self._stream_h:         # (the default stream's handle is 0)
            raise RuntimeError("phx: the current stream (0x%x) is not the stream this object was built on "
                               "(0x%x); run it outside torch.cuda.stream(...) or build it there"
                               % (cur, self._stream_h))

    def _pinned_small(self):
        """64 pinned host doubles, allocated once (small device reads)."""
        pin = getattr(self, "_pin_small", None)
        if pin is None:
            pin = self._pin_small = torch.empty(64, dtype=torch.float64, pin_memory=True)
        return pin

    def _read_small(self, t):
        """A few device doubles on the host: an async copy into a pinned buffer
        allocated once, then a wait on this object's stream (a pageable .cpu()
        stages through a bounce buffer: ~30-60 us more per read on the GPU)."""
        k = t.numel()
        if self.device.type != "cuda" or k > 64:
            return t.cpu().numpy()
        pin = self._pinned_small()
        self._check_stream()
        stream = torch.cuda.current_stream(self.device)
        pin[:k].copy_(t.reshape(-1), non_blocking=True)
        stream.synchronize()
        return pin[:k].numpy().copy()

    # ------------------------------------------------------------ host views
    def _bump(self):
        self._host_epoch += 1
        self._host_cache.clear()

    def _host(self, key):
        """numpy copy of a device array (cached until the next device op)."""
        if hasattr(self, "_settle"):
            self._settle()
        if key not in self._host_cache:
            S = self._S
            if key == "x":
                a = self._x.view(-1, S).cpu().numpy()
            elif key == "W":
                a = self._W.view(-1, S).cpu().numpy() if self.batch.nonant.N else np.zeros((0, S))
            elif key == "rho":
                a = self._rho.view(-1, S).cpu().numpy() if self.batch.nonant.N else np.zeros((0, S))
            elif key == "xbar":
                a = self._xbar_node.cpu().numpy()
            elif key == "xsqbar":
                a = self._xsqbar_node.cpu().numpy()
            elif key == "obj":
                a = (self._obj.cpu().numpy() + self._c0_int) * (1.0 if self.is_minimizing else -1.0)
            elif key == "outer":
                a = (self._outer.cpu().numpy() + self._c0_int) * (1.0 if self.is_minimizing else -1.0)
            elif key == "status":
                a = self._status.cpu().numpy()
            else:
                raise KeyError(key)
            self._host_cache[key] = a
        return self._host_cache[key]

    def _host_write(self, key, j, s, value):
        """write-through to the device array (W / rho mirrors)."""
        S = self._S
        if hasattr(self, "_settle"):
            self._settle()
        if key == "x":
            self._x_touched = True
        t = self._x if key == "x" else {"W": self._W, "rho": self._rho}[key]
        t[j * S + s] = float(value)
        if key in self._host_cache:
            self._host_cache[key][j, s] = float(value)
        if key == "x":
            self._conv_cache = None

    @property
    def spcomm(self):
        if self._spcomm is None:
            return None
        return self._spcomm()

    @spcomm.setter
    def spcomm(self, value):
        if self._spcomm is None:
            self._spcomm = weakref.ref(value)
        else:
            raise RuntimeError("SPBase.spcomm should only be set once")

    def _options_check(self, required_options, given_options):
        missing = [o for o in required_options if given_options.get(o) is None]
        if missing:
            raise ValueError("Missing the following required options: %s" % ", ".join(missing))

    # ------------------------------------------------------------ results
    def nonant_values(self):
        """(S_local, N) nonant values of the last solve (host copy)."""
        x = self._host("x")
        return x[self.batch.nonant.slot_col].T.copy()

    def gather_var_values_to_rank0(self, get_zero_prob_values=False):
        """{(scenario_name, var_name): value} of the nonants (spbase.py:547-581)."""
        xn = self.nonant_values()
        names = self.batch.nonant.var_names
        out = {}
        for k, sn in enumerate(self.local_scenario_names):
            for j, vn in enumerate(names):
                out[sn, vn] = float(xn[k, j])
        if self.n_proc == 1:
            return out
        res = self.mpicomm.gather(out, root=0)
        if self.cylinder_rank == 0:
            return {k: v for d in res for k, v in d.items()}
        return None

    def report_var_values_at_rank0(self, header="", print_zero_prob_values=False):
        vv = self.gather_var_values_to_rank0()
        if self.cylinder_rank == 0:
            if header:
                print(header)
            for (sn, vn), v in sorted(vv.items()):
                print("%s %s %.4f" % (sn, vn, v))


def ctypes_void():
    return ctypes.c_void_p()
