"""bench.py — PH scenario-iterations/s + time to conv < 1e-4 (BASELINE.json metric).

A "step" is one PH iteration over every scenario (Compute_Xbar -> Update_W ->
convergence_diff -> batched subproblem solve), the body of ``PHBase.iterk_loop``
(mpisppy/phbase.py:901-970).  Headline workload: farmer, crops_multiplier 1,
100,000 synthetic scenarios (BASELINE configs[2]; the metric is quoted on it and
it fits one MI355X), rho = 1, scenarios sharded contiguously over the ranks
(strong scaling: the 100k total is fixed).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU)

With --gpus N > 1 and no WORLD_SIZE in the environment, this process launches
the N ranks itself (torch.distributed.run, one process per GPU, 127.0.0.1
rendezvous) before it makes any GPU call, and exits with their exit code -- the
reference launches its ranks the same way (mpiexec -n N, examples/run_all.py:58-75).
--device cpu (test hook): gloo + the test-only host emulation of the C ABI
(tests/emu), no GPU call at all -- the launcher and the N-rank path run on CPU.

Metric: value = S (K + 1) / T, T = wall time of Iter0 + K PH
iterations (PHBase.Iter0 then PHBase.iterk_loop with PHIterLimit = K, on the
device: phx_iterk), bracketed by barrier + device synchronize (none in between:
Iter0's share from events around it), MAX over ranks; K
steps are timed, Iter0 counts as one more scenario-solve pass.  W warmup: a full
untimed Iter0 + W iterations on a separate PH object first (JIT, allocator).
Inputs resident in HBM before timing.  Extra keys:
  steady        S K / T_iterk (Iter0 excluded) and the per-iteration time
  conv_time     wall time from Iter0 to conv < 1e-4 (convthresh 1e-4), iterations
  roofline      the dominant kernel of the timed iterations (phx_lane_warm):
                algorithmic bytes / its average duration from HIP
                events recorded around it on the solve stream (sampled iterations)
  cpu_baseline  the oracle's CPU restatement of the reference PH (oracle/cpu_bench.py,
                one worker process per core) on a bounded sample, child process,
                rank 0 at N = 1
  configs       (N = 1) the other BASELINE configs, each timed the same way
                (Iter0 + K' iterations): C1 farmer x 3 (configs[0]), C3s8 farmer x
                12,500 (the 8-GPU per-rank slice of configs[2]), C3x1M farmer x
                1,000,000 (the over-cache HBM configuration), C2 farmer
                crops_multiplier=10 x 1,000, C4 aircond 10x10x10, C5a sslp_15_45 x
                10,000, C5b netdes network-50-30-H x 10,000 -- value, steady state,
                dominant kernel + roofline (+ PMC traffic and its ratio to the
                algorithmic bytes), CPU baseline (per-GPU share measured, whole host
                projected)
"""
import argparse
import gc
import json
import os
import subprocess
import sys
import time

_ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, _ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--build-after-warmup", action="store_true",
                    help="build the timed object after the warmup run (default: before it, so the warmup's "
                         "steps run right before the timed region)")
    ap.add_argument("--scens", type=int, default=100000)
    ap.add_argument("--cm", type=int, default=1)
    ap.add_argument("--rho", type=float, default=1.0)
    ap.add_argument("--lane-solver", type=int, default=1, help="1: structure-specialised lane solver first")
    ap.add_argument("--depth", type=int, default=4, help="phx_iterk: iterations kept enqueued ahead")
    ap.add_argument("--fused", type=int, default=1, help="phx_iterk: one launch per PH iteration")
    ap.add_argument("--kernel-timing-inline", action="store_true",
                    help="record the kernel-timing events in the metric's own timed run (round-5 form)")
    ap.add_argument("--timing-every", type=int, default=-5,
                    help="phx_iterk: T > 0: HIP events around the lane kernel of every T-th iteration; "
                         "T < 0: fused loop: one event pair around all its launches (back to back: no "
                         "per-launch event records in the timed loop), unfused: every |T|-th")
    ap.add_argument("--no-conv", action="store_true", help="skip time to conv < 1e-4")
    ap.add_argument("--conv-max-iters", type=int, default=10000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-scens", type=int, default=40000)
    ap.add_argument("--cpu-iters", type=int, default=6)
    ap.add_argument("--cpu-procs", type=int, default=16, help="worker processes (the GPU box's CPU share)")
    ap.add_argument("--cpu-samples", type=int, default=3, help="CPU baseline samples per config (median reported)")
    ap.add_argument("--configs", default="all", help="'all', 'none' or a comma list of C1,C3s8,C3x1M,C2,C4,C5a,C5b")
    ap.add_argument("--config-steps", type=int, default=10, help="K' of the other configs")
    ap.add_argument("--only", default=None, help="run one config as the headline (C2, C4, C5a, C5b)")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: test hook (gloo + the host emulation library, no GPU)")
    ap.add_argument("--so", default=None, help="extra solver options (JSON), e.g. '{\"seed_templates\": 0}'")
    ap.add_argument("--detail", default=os.path.join(_ROOT, "bench_detail.json"),
                    help="file for the full per-config record (stdout's last line is the compact headline)")
    ap.add_argument("--ar-probe", type=int, default=1,
                    help="N = 1: time phx_iterk with a no-op all-reduce callback (the per-iteration host "
                         "cost of the Python collective hook)")
    return ap.parse_args()


# ---------------------------------------------------------------- device plumbing
class Dev:
    """cuda: the GPU (RCCL for N > 1); cpu: the test hook (gloo, host emulation)."""

    def __init__(self, kind):
        self.kind = kind
        self.cuda = kind == "cuda"
        self.lib = None
        self.device = None
        if not self.cuda:
            from mpisppy_amd import _native
            self.lib = _native.Lib(os.path.join(_ROOT, "tests", "emu", "libphx_emu.so"), prefix="emu_phx_")
            self.device = "cpu"

    def sync(self):
        if self.cuda:
            torch.cuda.synchronize()

    def tensor(self, vals):
        return torch.tensor(vals, dtype=torch.float64, device="cuda" if self.cuda else "cpu")

    def empty_cache(self):
        if self.cuda:
            torch.cuda.empty_cache()


def launch_ranks(args):
    """--gpus N > 1 without WORLD_SIZE: start N ranks (one process per GPU) as
    children and return their exit code.  No GPU call happens in this process
    (importing torch does not initialise the GPU)."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % args.gpus,
           "--master-addr=127.0.0.1", "--master-port=%d" % port, os.path.abspath(__file__)] + sys.argv[1:]
    print("[bench] launching %d ranks: %s" % (args.gpus, " ".join(cmd)), file=sys.stderr, flush=True)
    return subprocess.run(cmd, env=env).returncode


# ---------------------------------------------------------------- algorithmic bytes
def lane_bytes(b, fused=False):
    """phx_lane_warm per scenario solve.  reads: varying A values, W
    and rho of the nonant slots with their x-bar index, the active-set words, plus
    c / bounds / row bounds where they vary; writes: x (n), row duals (m),
    objective, status + iteration count, flags, active-set words.  fused: + the
    previous nonant x and prob_coeff (Update_W / next x-bar), + the W write-back."""
    nw = (2 * (b.n + b.m) + 31) // 32
    rd = 8 * (b.nvar + 2 * b.nonant.N) + 4 * b.nonant.N + 4 * nw
    rd += 8 * b.n * int(b.c_vary) + 16 * b.n * int(b.bnd_vary) + 16 * b.m * int(b.rhs_vary)
    wr = 8 * (b.n + b.m + 1) + 4 * 5 + 4 * nw
    if fused:
        rd += 16 * b.nonant.N
        wr += 8 * b.nonant.N
    return rd + wr


def wg_bytes(b):
    """k_wg_warm per scenario solve: reads the varying A values, qN/pN of the nonant
    slots and the warm-start point (x n, y m); writes x, x0, xT (3n) and y, y0, yT
    (3m) plus status + iters."""
    return 8 * (b.nvar + 2 * b.nonant.N + b.n + b.m) + 8 * (3 * b.n + 3 * b.m) + 8


def sp_bytes(b):
    """k_sp_solve per scenario solve (phx_sp.h): reads the varying A values, c / bounds
    / row bounds where they vary, qN/pN of the nonant slots, the warm-start point
    (x n, y m); writes the outputs x (n), y (m) and the next warm start x, x0, xT,
    y, y0, yT, plus objective, status, iterations, flags."""
    rd = 8 * (b.nvar + 2 * b.nonant.N + b.n + b.m)
    rd += 8 * b.n * int(b.c_vary) + 16 * b.n * int(b.bnd_vary) + 16 * b.m * int(b.rhs_vary)
    wr = 8 * 4 * (b.n + b.m) + 8 + 12
    return rd + wr


# profiles/r*_pmc_<tag>_<kernel>.json of each secondary config (scripts/pmc_summary.py
# over the config's timed launches)
CONFIG_PMC_TAG = {"C3s8": "farmer12k5", "C2": "farmercm10_1k", "C4": "aircond1k", "C5a": "sslp10k", "C5b": "netdes10k",
                  "C3x1M": "farmer1m"}


def _current_source_hash(kernel):
    sys.path.insert(0, os.path.join(_ROOT, "scripts"))
    try:
        import src_hash
        return src_hash.source_hash(kernel)
    finally:
        sys.path.pop(0)


def pmc_traffic(kernel, tag):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC passes
    (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE; scripts/pmc_summary.py): counters
    need their own profiler runs, so they are read from profiles/ (newest first).
    Only a summary taken on the kernel's current sources counts (its
    source_sha256, scripts/src_hash.py): an older one is reported as stale and
    its bytes are not used.  Returns (bytes or None, file, status)."""
    import glob
    files = sorted(glob.glob(os.path.join(_ROOT, "profiles", "r*_pmc_%s_%s.json" % (tag, kernel))))
    if not files:
        return None, None, "no PMC summary"
    d = json.load(open(files[-1]))
    src = os.path.relpath(files[-1], _ROOT)
    cur = _current_source_hash(kernel)
    if d.get("source_sha256") is None or d.get("source_sha256") != cur:
        return None, src, "stale: measured on other %s sources (%s), current %s" % (
            kernel, (d.get("source_sha256") or "unrecorded")[:12], (cur or "?")[:12])
    return d.get("hbm_bytes_per_launch", {}).get("total"), src, "current (source_sha256 %s)" % cur[:12]


def valu_issue(kernel, tag, units, avg_s, lanes_per_wave=64, simds=1024, clock_hz=2.4e9):
    """The kernel's VALU-issue roofline from the committed SQ counter pass
    (profiles/r*_pmcsq_<tag>_<kernel>.json, same command, timed launches):
    SQ_INSTS_VALU wave-instructions per launch spread over the launch's
    wavefronts; the busiest SIMD holds ceil(waves / 1,024) of them, and a wave64
    VALU instruction issues in 4 cycles on a 16-lane SIMD (MI355X_MICROARCH.md:
    1,024 SIMDs, 2,400 MHz) -- the time the kernel would take if it issued a VALU
    instruction every cycle it could."""
    import glob
    files = sorted(glob.glob(os.path.join(_ROOT, "profiles", "r*_pmcsq_%s_%s.json" % (tag, kernel))))
    if not files or not avg_s:
        return None
    d = json.load(open(files[-1]))
    if d.get("source_sha256") is None or d.get("source_sha256") != _current_source_hash(kernel):
        return {"stale": True, "source": os.path.relpath(files[-1], _ROOT),
                "note": "SQ counters measured on other %s sources: not used" % kernel}
    insts = d.get("counters", {}).get("SQ_INSTS_VALU")
    if not insts:
        return None
    waves = -(-units // lanes_per_wave)
    per_wave = insts / waves
    busiest = -(-waves // simds)
    bound_s = busiest * per_wave * 4 / clock_hz
    return {"valu_insts_per_launch": insts, "valu_insts_per_wave": per_wave, "waves_per_launch": waves,
            "busiest_simd_waves": busiest, "issue_bound_us": bound_s * 1e6, "frac": bound_s / avg_s,
            "source": os.path.relpath(files[-1], _ROOT)}


def cpu_baseline(args, model="farmer", cm=1, scens=None, iters=None, total=None, timeout=900, procs=None):
    """oracle/cpu_bench.py in a child process (it never touches the GPU).

    Measured with P worker processes = the GPU box's CPU share per GPU (16: the
    pool's rule for worker pools on a one-GPU box), reported as
    ``per_gpu_share``.  ``whole_host`` is BASELINE.md's bar -- the reference
    under ``mpiexec -n P`` with P = all physical cores of the host -- projected
    from that measurement by perfect linear scaling over the physical cores
    (the subproblem solves are independent; the per-iteration reduction is a
    few doubles), which can only overstate the host: running ~128 worker
    processes on the box is outside its per-GPU CPU share."""
    procs = max(1, min(procs or args.cpu_procs, os.cpu_count() or 1))
    cmd = [sys.executable, "-m", "oracle.cpu_bench", "--model", model, "--scens", str(scens or args.cpu_scens),
           "--iters", str(iters or args.cpu_iters), "--procs", str(procs), "--cm", str(cm), "--rho", str(args.rho)]
    if total:
        cmd += ["--scens-total", str(total)]
    # several samples (each its own child process): the value is their median,
    # the spread their min / max (one short sample moved by 1.7x box to box, r05)
    runs = []
    for _ in range(max(1, args.cpu_samples)):
        try:
            r = subprocess.run(cmd, cwd=_ROOT, capture_output=True, text=True, timeout=timeout)
        except subprocess.TimeoutExpired:
            return {"error": "timeout"}
        if r.returncode != 0:
            return {"error": r.stderr[-500:]}
        runs.append(json.loads(r.stdout.strip().splitlines()[-1]))
    vals = sorted(x["value"] for x in runs)
    d = dict(runs[0])
    d["value"] = float(np.median(vals))
    d["seconds"] = float(np.median([x["seconds"] for x in runs]))
    out = {k: d[k] for k in ["value", "unit", "cores", "kind", "sample", "seconds", "host"]}
    out["spread"] = {"samples": len(vals), "min": vals[0], "median": d["value"], "max": vals[-1],
                     "values": vals, "stat": "median of the samples (each a fresh child process)"}
    host = d.get("host") or {}
    out["cpu_model"] = host.get("cpu_model")
    out["per_gpu_share"] = {"value": d["value"], "cores": d["cores"], "measured": True}
    phys = host.get("physical_cores")
    if phys:
        out["whole_host"] = {"value": d["value"] * phys / d["cores"], "cores": phys, "sockets": host.get("sockets"),
                             "measured": False,
                             "cap": "the GPU pool caps a one-GPU lease's worker pools at its CPU share (16 "
                                    "processes; nproc shows all %s CPUs): P = %d physical cores not runnable here"
                                    % (host.get("nproc"), phys),
                             "how": "per_gpu_share x physical cores / %d (perfect linear scaling: an upper bound "
                                    "on the host)" % d["cores"]}
    return out


# ---------------------------------------------------------------- workloads
def workloads():
    from mpisppy_amd.examples import farmer, sslp, netdes, aircond
    from mpisppy_amd.utils import sputils
    bfs = [10, 10, 10]
    return {
        "C1": dict(creator=farmer.scenario_creator, names=lambda S: farmer.scenario_names_creator(3),
                   kw=lambda S, cm: {"num_scens": 3, "crops_multiplier": 1}, nodes=None, S=3,
                   desc="farmer crops_multiplier=1, 3 scenarios, rho=1 (BASELINE configs[0]; the reference runs it "
                        "under mpiexec -n 3)",
                   cpu=dict(model="farmer", cm=1, scens=3, iters=100, total=3, procs=3)),
        "C3": dict(creator=farmer.scenario_creator, names=lambda S: farmer.scenario_names_creator(S),
                   kw=lambda S, cm: {"num_scens": S, "crops_multiplier": cm}, nodes=None,
                   desc="farmer crops_multiplier=%d, %d scenarios (BASELINE configs[2])"),
        "C3s8": dict(creator=farmer.scenario_creator, names=lambda S: farmer.scenario_names_creator(12500),
                     kw=lambda S, cm: {"num_scens": 12500, "crops_multiplier": 1}, nodes=None, S=12500, K=20,
                     desc="farmer crops_multiplier=1, 12,500 scenarios on one GPU (the per-rank slice of "
                          "configs[2] on 8 GPUs: 100,000 / 8)",
                     cpu="headline"),
        "C3x1M": dict(creator=farmer.scenario_creator, names=lambda S: farmer.scenario_names_creator(1000000),
                      kw=lambda S, cm: {"num_scens": 1000000, "crops_multiplier": 1}, nodes=None, S=1000000,
                      desc="farmer crops_multiplier=1, 1,000,000 scenarios on one GPU (the over-cache HBM "
                           "configuration of configs[2]: working set > 256 MiB Infinity Cache)",
                      cpu="headline"),
        "C2": dict(creator=farmer.scenario_creator, names=lambda S: farmer.scenario_names_creator(1000),
                   kw=lambda S, cm: {"num_scens": 1000, "crops_multiplier": 10}, nodes=None, S=1000,
                   desc="farmer crops_multiplier=10, 1,000 scenarios (BASELINE configs[1])",
                   # the workgroup pass's round budget: the lanes that need more
                   # go on to the sparse interior point either way (measured,
                   # r04_s31/s32: 16 rounds 0.98-0.99 ms per step, 8 0.94-0.95,
                   # 6 0.92, 4 2.76 -- eight stops instead of one; r05_s24, the
                   # in-stream sparse step: 8 0.604, 6 0.602, 4 1.88); in the first
                   # PH iteration after Iter0 the pass certifies almost no lane
                   # (emulation, 300 scenarios: 12 of 300 with 8 rounds), so one
                   # round there (wg_first) before the interior point
                   so={"wg_warm": 8, "wg_first": 1},
                   cpu=dict(model="farmer", cm=10, scens=1000, iters=8, total=1000)),
        "C4": dict(creator=aircond.scenario_creator, names=lambda S: ["scen%d" % i for i in range(1000)],
                   kw=lambda S, cm: {"branching_factors": bfs}, S=1000,
                   nodes=sputils.create_nodenames_from_branching_factors(bfs),
                   desc="aircond branching 10x10x10, 1,000 scenarios, 111 non-leaf nodes (BASELINE configs[3])",
                   # every timed launch bracketed (the unfused loop's default samples
                   # every fifth: two of ten, and C4's launches range 25-190 us with
                   # the early iterations' rescue rounds -- r04 verdict): the average
                   # is the timed window's, as a kernel trace's.  The event records
                   # themselves cost the stream ~6 us on each side of every launch
                   # (r06 s9 trace), so they run in a second timed run of their own:
                   # the metric's run records none
                   kernel_timing={"iterk_timing": -1},
                   # bounded multi-change active-set updates (every violation within
                   # 0.2 of the worst, 4 rounds, then single changes): the early
                   # iterations' rescue tails on 1-3 lanes set phx_lane_all's time --
                   # steady step 0.121 / 0.121 -> 0.111 / 0.110 ms over two pairs on one
                   # box (r06 s20); theta 0.1 / 0.3 and 2 / 3 / 6 rounds 0.114-0.122
                   # (r06 s22).  On farmer the same setting costs 6 % (headline) to
                   # 14 % (C3s8), so it is this problem's option, not a default
                   so={"lane_multi_theta": 0.2, "lane_multi_rounds": 4},
                   cpu=dict(model="aircond", scens=1000, iters=40, total=1000)),
        "C5a": dict(creator=sslp.scenario_creator, names=lambda S: sslp.scenario_names_creator(10000),
                    kw=lambda S, cm: {"num_scens": 10000}, nodes=None, S=10000,
                    desc="sslp_15_45 LP relaxation, 10,000 stochastic-RHS scenarios (BASELINE configs[4])",
                    # a few sslp lanes need the sparse interior point in every PH
                    # iteration anyway: more workgroup rounds only delay them
                    # (measured: 16 rounds 24.4, 8 18.9, 4 16.3 ms per iteration;
                    # profiles/r02_s18_wg_rounds.txt)
                    so={"wg_warm": 4},
                    cpu=dict(model="sslp", scens=512, iters=2, total=10000)),
        "C5b": dict(creator=netdes.scenario_creator, names=lambda S: netdes.scenario_names_creator(10000),
                    kw=lambda S, cm: {"instance": "network-50-30-H-01", "num_scens": 10000}, nodes=None, S=10000,
                    desc="netdes network-50-30-H LP relaxation, 10,000 scenarios (BASELINE configs[4])",
                    cpu=dict(model="netdes50", scens=128, iters=4, total=10000)),
    }


def make_ph(w, S, cm, rho, so, iters, dev, convthresh=1e-10, cls=None):
    from mpisppy_amd.opt.ph import PH
    opts = {"solver_name": "phx", "PHIterLimit": iters, "defaultPHrho": rho, "convthresh": convthresh,
            "verbose": False, "display_progress": False, "iter0_solver_options": dict(so),
            "iterk_solver_options": dict(so)}
    return (cls or PH)(opts, w["names"](S), w["creator"], scenario_creator_kwargs=w["kw"](S, cm),
                       all_nodenames=w["nodes"], _native_lib=dev.lib, _device=dev.device)


def timed_run(ph, K, dev):
    """Iter0 + K PH iterations, bracketed by barrier + synchronize (PH.ph_main without
    post_loops).  Returns (T, T_iter0, T_iterk), the max over ranks."""
    ph.PH_Prep()
    ph.subproblem_creation(False)
    ph.options["PHIterLimit"] = K
    # Python's cyclic garbage collector off inside the timed region (as timeit
    # does): a generation-2 collection over the process's objects (torch's among
    # them) stalled the host ~13 ms inside the region on some runs -- 7-14e7
    # instead of ~1.9e9 (r06 s23 / s24) -- with the GPU idle behind it.  The
    # full collection itself runs before the warm-up (gc_settle), not here: its
    # walk over every object leaves the host's caches cold for the region.  No
    # work of the path is skipped: the collector frees nothing the path allocates
    with no_gc():
        return _timed_region(ph, dev)


def gc_settle():
    """A full collection, then every surviving object frozen (gc.freeze: later
    collections skip them) -- before a warm-up, outside any timed region."""
    if os.environ.get("PHX_BENCH_GC") == "1":
        return
    gc.collect()
    gc.freeze()


class no_gc:
    """The cyclic collector off until exit (timed regions).  PHX_BENCH_GC=1 leaves
    it on (A/B runs)."""

    def __enter__(self):
        self.was = gc.isenabled()
        if os.environ.get("PHX_BENCH_GC") != "1":
            gc.disable()
        return self

    def __exit__(self, *exc):
        if self.was:
            gc.enable()
        return False


def _timed_region(ph, dev):
    ph.mpicomm.Barrier()
    dev.sync()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)] if dev.cuda else None
    t0 = time.perf_counter()
    if ev:
        ev[0].record()
    ph._defer_iter0_checks = True          # as PH.ph_main does
    ph.Iter0()
    # (no synchronize between Iter0 and iterk_loop -- ph_main has none: the
    # Iter0 share is the device time between two events on the same stream,
    # its last work included)
    if ev:
        ev[1].record()
    else:
        t1 = time.perf_counter()
    ph.iterk_loop()
    ph._settle()
    dev.sync()
    ph.mpicomm.Barrier()
    t2 = time.perf_counter()
    if ev:
        t1 = t0 + ev[0].elapsed_time(ev[1]) / 1e3
    tt = dev.tensor([t2 - t0, t1 - t0, t2 - t1])
    ph.mpicomm.allreduce_max_(tt)
    return [float(v) for v in tt.cpu()]


def final_state(ph):
    """The run's x-bar / conv (rank-independent: all-reduced), for checks of the N-rank path."""
    xb = ph.xbar_by_node()
    return {"xbar": {nd: [float(v) for v in a[0]] for nd, a in list(xb.items())[:4]}, "conv": ph.conv,
            "trivial_bound": ph.trivial_bound}


def ar_probe(w, S, cm, rho, so, K, dev):
    """Host cost of the Python all-reduce hook of phx_iterk: the same K iterations
    on one rank with and without a no-op callback installed (the multi-rank path
    of phx_iterk: one or two callbacks per iteration, enqueued ahead of the GPU).
    Returns the steady per-iteration times and the callback's own host time."""
    from mpisppy_amd import _native
    from mpisppy_amd.opt.ph import PH
    calls = [0, 0.0]

    class NoopPH(PH):
        def _iterk_argstruct(self):
            a = super()._iterk_argstruct()
            if not getattr(self, "_noop_cb", None):
                def cb(user, ptr, count, stream):
                    t = time.perf_counter()
                    calls[0] += 1
                    calls[1] += time.perf_counter() - t
                    return 0
                self._noop_cb = _native.ALLREDUCE_FN(cb)
                a.allreduce = self._noop_cb
            return a

    out = {}
    variants = [("without", PH, so), ("noop_callback", NoopPH, so)]
    if dev.cuda:
        # the N > 1 path with phx_iterk's own RCCL all-reduce (one-rank communicator)
        variants.append(("rccl_in_loop_1rank", PH, dict(so, native_comm=2)))
    for name, cls, sov in variants:
        ph = make_ph(w, S, cm, rho, sov, K, dev, cls=cls)
        T, T0, Tk = timed_run(ph, K, dev)
        out[name] = {"ms_per_iter": Tk * 1e3 / K, "fused": bool(getattr(ph, "iterk_stats", {}).get("fused"))}
        del ph
        dev.empty_cache()
    out["callbacks"] = calls[0]
    out["callbacks_per_iter"] = calls[0] / K
    out["delta_us_per_iter"] = (out["noop_callback"]["ms_per_iter"] - out["without"]["ms_per_iter"]) * 1e3
    if "rccl_in_loop_1rank" in out:
        out["rccl_delta_us_per_iter"] = (out["rccl_in_loop_1rank"]["ms_per_iter"]
                                         - out["without"]["ms_per_iter"]) * 1e3
    out["note"] = ("a no-op ctypes callback on one rank (the N > 1 kernel path: conv test after the "
                   "all-reduce) vs phx_iterk's own ncclAllReduce on a one-rank communicator (the default "
                   "for N > 1 on GPUs); a real N-rank collective adds its xGMI latency")
    return out


def dominant_kernel(ph, K, fused):
    """(kernel, avg launch seconds, launches, bytes per unit, units per launch) of the
    timed iterations' dominant kernel."""
    b = ph.batch
    st = getattr(ph, "iterk_stats", None)
    if st is not None and st.get("warm_launches", 0) > 0:
        # phx_iterk times its per-iteration solve kernel: the lane solver's warm
        # launch, or (subproblems above the lane limits) the workgroup pass
        info = ph._native.jit_info(ph._ctx).decode()
        if info.startswith("on"):
            # the lane kernel that ran (phx_kernels.hip enqueue_lane_solve): the
            # fused iteration kernel (its one-wave-per-SIMD build for batches of
            # at most one wavefront per SIMD), or unfused (multistage) the one-launch
            # small-batch solve / the warm pass
            small = -(-b.S // 64) <= simds()
            if st.get("fused"):
                # (the one-wave build at every size unless PHX_FZ2=1, phx_kernels.hip)
                fz2 = os.environ.get("PHX_FZ2") == "1"
                kname = "phx_lane_warm_fz" if (fz2 and not small) else "phx_lane_warm_fz1"
                # (above one wavefront per SIMD the two-wave build, unless PHX_FZR2=0)
                if not small and not fz2 and os.environ.get("PHX_FZR2") != "0":
                    kname = "phx_lane_warm_fzr2"
                # (the compacting build, phx_kernels.hip, opt-in PHX_FZC=1)
                if os.environ.get("PHX_FZC") == "1" and os.environ.get("PHX_FZ_LEGACY") != "1":
                    kname = "phx_lane_warm_fzc"
            else:
                kname = "phx_lane_all" if small else "phx_lane_warm"
                # (the build that re-loads per round where the register build spills)
                if small and "all=reload" in info:
                    kname = "phx_lane_all_rl"
                elif small and "all=park" in info:
                    kname = "phx_lane_all_pk"
            return (kname, st["lane_warm_ms"] / 1e3 / st["warm_launches"], st["warm_launches"],
                    lane_bytes(b, fused=bool(st.get("fused")) and fused), b.S)
        if "workgroup solver on" in info:
            return ("k_wg_warm", st["lane_warm_ms"] / 1e3 / st["warm_launches"], st["warm_launches"], wg_bytes(b),
                    b.S)
        # the sparse solver's warm pass (the bracketed events also cover its
        # PH-term and warm-start kernels: a few us against tens of ms)
        return ("k_sp_solve", st["lane_warm_ms"] / 1e3 / st["warm_launches"], st["warm_launches"], sp_bytes(b), b.S)
    stats = ph.solve_stats[-K:]
    cand = {
        "phx_lane_warm": (sum(s.get("lane_warm_ms", 0.0) for s in stats), lane_bytes(b)),
        "k_wg_warm": (sum(s.get("wg_ms", 0.0) for s in stats), wg_bytes(b)),
        "k_sp_solve": (sum(s.get("sp_ms", 0.0) for s in stats), sp_bytes(b)),
    }
    name = max(cand, key=lambda k: cand[k][0])
    ms, bpu = cand[name]
    launches = sum(1 for s in stats if s.get({"phx_lane_warm": "lane_warm_ms", "k_wg_warm": "wg_ms",
                                              "k_sp_solve": "sp_ms"}[name], 0.0) > 0.0)
    units = b.S
    if name == "k_sp_solve":
        # the sparse pass after the dense warm pass sees only the lanes that pass left
        cert = [s.get("sp_certified", 0) for s in stats if s.get("sp_ms", 0.0) > 0.0]
        if cert and any(s.get("wg_ms", 0.0) > 0.0 for s in stats):
            units = max(1, int(np.mean(cert)))
    return name, ms / 1e3 / max(launches, 1), launches, bpu, units


def simds():
    """SIMDs of the GPU (4 per CU), the lane kernels' one-wave slots."""
    try:
        return 4 * torch.cuda.get_device_properties(0).multi_processor_count
    except Exception:
        return 1024


def roofline(kernel, avg_s, launches, bpu, units, traffic=None, traffic_src=None, traffic_status=None):
    bytes_per_launch = bpu * units
    achieved = bytes_per_launch / avg_s / 1e9 if avg_s > 0 else 0.0
    return {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_unit": "bytes/launch",
            "traffic_source": traffic_src, "traffic_status": traffic_status,
            "traffic_ratio": (traffic / bytes_per_launch) if (traffic and bytes_per_launch) else None,
            "algorithmic_bytes_per_launch": bytes_per_launch, "kernel": kernel,
            "bytes_per_unit": bpu, "unit_def": "scenario solve", "units_per_launch": units,
            "avg_launch_us": avg_s * 1e6, "launches": launches,
            "launch_timing": LAUNCH_TIMING.get(kernel, "HIP events around sampled launches")}


# how phx_iterk's events time the dominant kernel (bench --timing-every < 0)
LAUNCH_TIMING = {k: ("one HIP event pair around all the fused launches of the timed loop (back to back on "
                     "phx_iterk's stream; no per-launch records in between)")
                 for k in ("phx_lane_warm_fz", "phx_lane_warm_fz1", "phx_lane_warm_fzc", "phx_lane_warm_fzr2")}


def run_config(name, w, args, K, so, world, dev):
    """One secondary config at N = 1: Iter0 + K iterations on a fresh PH object."""
    S = w["S"]
    so = dict(so, **w.get("so", {}))
    # warmup as the headline's: an untimed Iter0 + W iterations on its own
    # object (each kernel's first launch -- code object load, the queue's
    # scratch growth -- outside the timed run)
    if args.warmup > 0:
        gc_settle()
        ph = make_ph(w, S, 1, args.rho, so, args.warmup, dev)
        ph.ph_main(finalize=False)
        dev.sync()
        del ph
    ktim = w.get("kernel_timing")
    if ktim:
        so = dict(so, iterk_timing=0)      # the metric's run: no event records in the loop
    t = time.perf_counter()
    ph = make_ph(w, S, 1, args.rho, so, K, dev)
    dev.sync()
    setup = time.perf_counter() - t
    T, T0, Tk = timed_run(ph, K, dev)
    if ktim:
        # the dominant kernel's launches timed in a run of their own (same data, same K)
        phk = make_ph(w, S, 1, args.rho, dict(so, **ktim), K, dev)
        timed_run(phk, K, dev)
        kernel, avg_s, launches, bpu, units = dominant_kernel(phk, K, True)
        del phk
    else:
        kernel, avg_s, launches, bpu, units = dominant_kernel(ph, K, True)
    nbad = sum(s.get("not_optimal", 0) for s in ph.solve_stats)
    st = getattr(ph, "iterk_stats", None)
    if st is not None:
        nbad += st.get("not_optimal", 0)
    res = {"workload": w["desc"], "scenarios": S, "n": ph.batch.n, "m": ph.batch.m, "nnz": ph.batch.nnz,
           "nonants": ph.batch.nonant.N, "steps": K,
           "value": S * (K + 1) / T, "unit": "scenario-iterations/s", "T_s": T, "iter0_s": T0,
           "steady": {"value": S * K / Tk, "ms_per_step": Tk * 1e3 / K},
           "roofline": roofline(kernel, avg_s, launches, bpu, units,
                                *pmc_traffic(kernel, CONFIG_PMC_TAG.get(name, name))),
           "solver": ph._native.jit_info(ph._ctx).decode(), "not_optimal": nbad, "setup_s": setup,
           "loop": "phx_iterk (device-driven)" if st is not None else "PHBase host loop (deferred solves)",
           "iterk": ({k: st.get(k) for k in ("iters", "fused", "straggler_stops", "stragglers", "warm_launches")}
                     if st is not None else None),
           "solver_options": w.get("so", {})}
    if w.get("cpu") and not args.no_cpu_baseline:
        c = w["cpu"]
        if c == "headline":
            # the same subproblems (farmer cm=1) as the headline: its baseline
            hb = getattr(args, "_headline_cpu", None)
            res["cpu_baseline"] = dict(hb, note="the headline's (same farmer cm=1 subproblems)") if hb else None
        else:
            res["cpu_baseline"] = cpu_baseline(args, model=c["model"], cm=c.get("cm", 1), scens=c["scens"],
                                               iters=c["iters"], total=c["total"], procs=c.get("procs"))
    del ph
    dev.empty_cache()
    return res


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print("[bench] --gpus %d but WORLD_SIZE=%d: running %d ranks" % (args.gpus, world, world),
              file=sys.stderr, flush=True)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.device == "cuda":
            torch.cuda.set_device(local_rank)
        dist.init_process_group(backend="nccl" if args.device == "cuda" else "gloo")
    elif args.device == "cuda":
        torch.cuda.set_device(0)
    import mpisppy_amd  # noqa: F401
    dev = Dev(args.device)
    W = workloads()
    K = args.steps
    so = {"lane_solver": args.lane_solver, "iterk_depth": args.depth, "iterk_timing": args.timing_every,
          "iterk_fused": args.fused}
    hl = W["C3"] if args.only is None else W[args.only]
    so.update(hl.get("so", {}))
    if args.so:
        so.update(json.loads(args.so))
    S = args.scens if args.only is None else hl["S"]
    cm = args.cm if args.only is None else 1
    # the metric's run records no events in its loop: the dominant kernel's
    # launches are timed by phx_iterk's events in a second timed run of their own
    # (same data, same K) -- each event record costs the stream ~6 us (r06 s27
    # trace: the window's two records, 6.5 + 6.1 us of idle stream inside T);
    # --kernel-timing-inline: the round-5 form, events in the metric's run
    ktim = args.timing_every != 0 and not args.kernel_timing_inline
    so_metric = dict(so, iterk_timing=0) if ktim else so
    # ---- the timed run's object (setup: outside the timed region) ----
    def build_timed():
        t = time.perf_counter()
        obj = make_ph(hl, S, cm, args.rho, so_metric, K, dev)
        dev.sync()
        return obj, time.perf_counter() - t
    if not args.build_after_warmup:
        ph_timed, t_setup = build_timed()
    # ---- warmup: a full untimed Iter0 + W iterations on its own object, right
    # before the timed region (the GPU does not idle between them while the
    # timed object is built) ----
    t = time.perf_counter()
    gc_settle()
    ph = make_ph(hl, S, cm, args.rho, so, args.warmup, dev)
    print("[bench] warmup object built (%.1f s)" % (time.perf_counter() - t), file=sys.stderr, flush=True)
    ph.ph_main(finalize=False)
    dev.sync()
    t_warm = time.perf_counter() - t
    print("[bench] warmup done (%.1f s)" % t_warm, file=sys.stderr, flush=True)
    del ph
    # ---- timed: Iter0 + K iterations on a fresh object ----
    if args.build_after_warmup:
        ph_timed, t_setup = build_timed()
    ph = ph_timed
    del ph_timed
    T, T0, Tk = timed_run(ph, K, dev)
    print("[bench] timed run done (%.3f ms)" % (T * 1e3), file=sys.stderr, flush=True)
    st = getattr(ph, "iterk_stats", None)
    if st is not None and (st["iters"] != K or st["solves"] != K):
        raise RuntimeError("timed iterk_loop did not run %d full iterations: %s" % (K, st))
    if ktim:
        phk = make_ph(hl, S, cm, args.rho, so, K, dev)
        dev.sync()
        timed_run(phk, K, dev)
        kernel, avg_s, launches, bpu, units = dominant_kernel(phk, K, args.fused)
        del phk
    else:
        kernel, avg_s, launches, bpu, units = dominant_kernel(ph, K, args.fused)
    b = ph.batch
    if world != 1:
        traffic, tsrc, tstat = None, None, "N > 1: per-rank PMC not collected"
    elif args.only is not None:
        traffic, tsrc, tstat = pmc_traffic(kernel, CONFIG_PMC_TAG.get(args.only, args.only))
    else:
        traffic, tsrc, tstat = (pmc_traffic(kernel, "farmer100k") if S == 100000 and cm == 1
                                else (None, None, "no PMC summary for this size"))
    nbad = sum(s.get("not_optimal", 0) for s in ph.solve_stats) + (st.get("not_optimal", 0) if st else 0)
    res = {
        "metric": "PH scenario-iterations/sec (farmer 100k) + time to conv<1e-4",
        "value": S * (K + 1) / T,
        "unit": "scenario-iterations/s",
        "n_gpus": world,
        "steps": K,
        "warmup": args.warmup,
        "ms_per_step": T * 1e3 / (K + 1),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (the reference's scenario generators restated: RandomState-seeded yields etc.)",
        "config": {"workload": (hl["desc"] % (cm, S)) if args.only is None else hl["desc"],
                   "scenarios": S, "scenarios_per_gpu": b.S, "n": b.n, "m": b.m, "nnz": b.nnz,
                   "nnz_varying": b.nvar, "nonants": b.nonant.N, "rho": args.rho,
                   "timed": "Iter0 + K PH iterations (value = S(K+1)/T, SURVEY §8(d))",
                   "parallelism": "scenario-sharded x%d, RCCL allreduce" % world},
        "T_s": T, "iter0_s": T0,
        "steady": {"value": S * K / Tk, "ms_per_step": Tk * 1e3 / K, "def": "S K / T_iterk (Iter0 excluded)"},
        "roofline": dict(roofline(kernel, avg_s, launches, bpu, units, traffic, tsrc, tstat),
                         valu=valu_issue(kernel, "farmer100k", units, avg_s, simds=simds())
                         if (world == 1 and args.only is None and S == 100000 and cm == 1) else None,
                         timing_run=("a second timed run of the same K (the metric's run records no events)"
                                     if ktim else "the metric's run")),
        "loop": ("PHBase.iterk_loop -> phx_iterk (device-driven, depth %d%s)"
                 % (args.depth, ", fused" if st and st.get("fused") else "")) if st else "PHBase host loop",
        "not_optimal": nbad, "setup_s": t_setup, "warmup_s": t_warm,
        "iterk": ({k: st.get(k) for k in ("iters", "fused", "straggler_stops", "stragglers", "warm_launches")}
                  if st else None),
        "solver": ph._native.jit_info(ph._ctx).decode(),
        "final": final_state(ph),
    }
    if args.device == "cpu":
        res["device"] = "cpu (test hook: gloo + host emulation library; not a measurement)"
    del ph
    dev.empty_cache()
    # ---- time to conv < 1e-4 from Iter0 (fresh object, same data) ----
    if not args.no_conv:
        ph2 = make_ph(hl, S, cm, args.rho, so_metric, args.conv_max_iters, dev, convthresh=1e-4)
        dev.sync()
        with no_gc():                       # (as the timed run)
            ph2.mpicomm.Barrier()
            t0 = time.perf_counter()
            ph2.ph_main(finalize=False)
            dev.sync()
            tc = dev.tensor([time.perf_counter() - t0])
        ph2.mpicomm.allreduce_max_(tc)
        res["conv_time"] = {"seconds": float(tc.item()), "iterations": ph2._PHIter, "conv": ph2.conv,
                            "convthresh": 1e-4, "converged": bool(ph2.conv is not None and ph2.conv < 1e-4)}
        del ph2
        dev.empty_cache()
    # ---- host cost of the Python all-reduce hook (one rank) ----
    if world == 1 and args.only is None and args.ar_probe:
        res["allreduce_hook"] = ar_probe(hl, S, cm, args.rho, so, K, dev)
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.only is None:
        res["cpu_baseline"] = cpu_baseline(args, cm=cm)
        args._headline_cpu = res["cpu_baseline"]
    # ---- the other BASELINE configs (one GPU) ----
    if world == 1 and args.only is None and args.configs != "none":
        names = (["C1", "C3s8", "C3x1M", "C2", "C4", "C5a", "C5b"] if args.configs == "all"
                 else args.configs.split(","))
        res["configs"] = {}
        for nm in names:
            try:
                res["configs"][nm] = run_config(nm, W[nm], args, W[nm].get("K", min(K, args.config_steps)), so,
                                                world, dev)
            except Exception as e:     # reported, never hidden
                res["configs"][nm] = {"error": repr(e)[:500]}
            print("[bench] %s done" % nm, file=sys.stderr, flush=True)
    if rank == 0:
        # the full record (every config's workload, solver, PMC provenance, CPU
        # sample text) goes to a file; stdout's LAST line is the compact headline
        # the driver parses (<= LINE_CAP bytes; stderr stays short too: the
        # driver keeps only the tail of both)
        full = json.dumps(res)
        try:
            with open(args.detail, "w") as f:
                f.write(full + "\n")
            print("[bench] full record: %s (%d bytes)" % (args.detail, len(full)), file=sys.stderr, flush=True)
        except OSError as e:
            print("[bench] could not write %s: %r" % (args.detail, e), file=sys.stderr, flush=True)
        print(json.dumps(compact_line(res, args.detail)), flush=True)
    if world > 1:
        dist.destroy_process_group()


LINE_CAP = 8000     # bytes of the stdout headline line (the driver's parser: <= 8 KB)


def _r(v, nd=4):
    """Round a float to nd significant digits (compact line); other values as is."""
    if isinstance(v, float):
        return float("%.*g" % (nd, v))
    return v


def _roof_short(rf, full=True):
    if not rf:
        return None
    keys = (["bound", "achieved", "peak", "unit", "frac", "traffic", "traffic_ratio", "kernel", "bytes_per_unit",
             "units_per_launch", "algorithmic_bytes_per_launch", "avg_launch_us", "launches"] if full
            else ["kernel", "frac", "traffic_ratio", "avg_launch_us"])
    out = {k: _r(rf.get(k)) for k in keys if k in rf}
    if full:
        out["traffic_unit"] = "bytes/launch"
        out["traffic_source"] = rf.get("traffic_source")
        st = rf.get("traffic_status") or ""
        out["traffic_current"] = st.startswith("current")
        if rf.get("timing_run"):
            out["timing_run"] = rf["timing_run"]
        v = rf.get("valu")
        if isinstance(v, dict) and not v.get("stale"):
            out["valu"] = {k: _r(v.get(k)) for k in ("valu_insts_per_wave", "waves_per_launch", "busiest_simd_waves",
                                                   "issue_bound_us", "frac", "source")}
    return out


def _cpu_short(cb, full=True):
    if not cb or "value" not in cb:
        return cb
    out = {"value": _r(cb["value"]), "unit": cb.get("unit"), "cores": cb.get("cores"), "kind": cb.get("kind")}
    sp = cb.get("spread")
    if sp:
        out["spread"] = {"samples": sp.get("samples"), "min": _r(sp.get("min")), "max": _r(sp.get("max"))}
    if full:
        out["sample"] = (cb.get("sample") or "")[:240]
        out["seconds"] = _r(cb.get("seconds"))
        out["cpu_model"] = cb.get("cpu_model")
        wh = cb.get("whole_host")
        if wh:
            out["whole_host"] = {k: _r(wh.get(k)) for k in ("value", "cores", "measured", "cap", "how") if k in wh}
            if isinstance(out["whole_host"].get("how"), str):
                out["whole_host"]["how"] = out["whole_host"]["how"][:200]
        if cb.get("scaling"):
            out["scaling"] = cb["scaling"]
    return out


def compact_line(res, detail_path):
    """The driver-readable headline: BASELINE's metric and the contract keys, the
    dominant kernel's roofline (traffic, ratio, VALU issue), the CPU baseline,
    conv_time, Iter0 / steady, and per config value / ms_per_step / frac /
    traffic_ratio / CPU value / avg_launch_us.  Everything else is in the detail
    file.  Falls back to fewer keys if a field ever makes it longer than LINE_CAP."""
    keep = ["metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data"]
    out = {k: _r(res[k], 6) if k in ("value", "ms_per_step") else res[k] for k in keep if k in res}
    c = res.get("config", {})
    out["config"] = {k: c.get(k) for k in ("workload", "scenarios", "scenarios_per_gpu", "n", "m", "nonants", "rho",
                                           "parallelism") if k in c}
    out["T_s"] = _r(res.get("T_s"), 5)
    out["iter0_s"] = _r(res.get("iter0_s"), 4)
    st = res.get("steady") or {}
    out["steady"] = {"value": _r(st.get("value")), "ms_per_step": _r(st.get("ms_per_step"))}
    out["roofline"] = _roof_short(res.get("roofline"))
    if "cpu_baseline" in res:
        out["cpu_baseline"] = _cpu_short(res["cpu_baseline"])
    if "conv_time" in res:
        ct = res["conv_time"]
        out["conv_time"] = {"seconds": _r(ct.get("seconds")), "iterations": ct.get("iterations"),
                            "converged": ct.get("converged"), "convthresh": ct.get("convthresh")}
    if res.get("iterk"):
        out["iterk"] = res["iterk"]
    out["not_optimal"] = res.get("not_optimal")
    if "device" in res:
        out["device"] = res["device"]
    if "final" in res:
        f = res["final"]
        out["final"] = {"xbar": f.get("xbar"), "conv": f.get("conv"), "trivial_bound": f.get("trivial_bound")}
    if res.get("configs"):
        cs = {}
        for nm, cr in res["configs"].items():
            if "error" in cr:
                cs[nm] = {"error": cr["error"][:120]}
                continue
            cst = cr.get("steady") or {}
            rf = cr.get("roofline") or {}
            cb = cr.get("cpu_baseline") or {}
            cs[nm] = {"S": cr.get("scenarios"), "value": _r(cr.get("value")), "ms_per_step": _r(cst.get("ms_per_step")),
                      "iter0_s": _r(cr.get("iter0_s"), 3), "kernel": rf.get("kernel"), "frac": _r(rf.get("frac"), 3),
                      "traffic_ratio": _r(rf.get("traffic_ratio"), 3), "avg_launch_us": _r(rf.get("avg_launch_us")),
                      "cpu": _r(cb.get("value")) if isinstance(cb, dict) else None,
                      "cpu_spread": ([_r((cb.get("spread") or {}).get("min")), _r((cb.get("spread") or {}).get("max"))]
                                     if isinstance(cb, dict) and cb.get("spread") else None),
                      "stops": (cr.get("iterk") or {}).get("straggler_stops"), "not_optimal": cr.get("not_optimal")}
        out["configs"] = cs
    out["detail"] = os.path.relpath(detail_path, _ROOT) if os.path.isabs(detail_path) else detail_path
    line = json.dumps(out)
    # shed the least important fields if the line ever outgrows the cap
    for drop in (("final",), ("iterk",), ("configs",)):
        if len(line.encode()) <= LINE_CAP:
            break
        for k in drop:
            out.pop(k, None)
        line = json.dumps(out)
    if len(line.encode()) > LINE_CAP and out.get("cpu_baseline"):
        out["cpu_baseline"] = _cpu_short(res["cpu_baseline"], full=False)
        line = json.dumps(out)
    if len(line.encode()) > LINE_CAP:
        # last resort: the contract keys (and the two objects) in their short forms
        out = {k: out[k] for k in keep + ["config"] if k in out}
        out["roofline"] = _roof_short(res.get("roofline"), full=False)
        if isinstance(res.get("cpu_baseline"), dict) and "value" in res["cpu_baseline"]:
            out["cpu_baseline"] = _cpu_short(res["cpu_baseline"], full=False)
        line = json.dumps(out)
    if len(line.encode()) > LINE_CAP:
        out.pop("config", None)
        out["data"] = "synthetic"
        line = json.dumps(out)
    assert len(line.encode()) <= LINE_CAP, len(line.encode())
    return out


if __name__ == "__main__":
    main()
