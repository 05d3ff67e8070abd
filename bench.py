"""bench.py — PH scenario-iterations/s on farmer (BASELINE.json metric).

A "step" is one PH iteration over every scenario (Compute_Xbar -> Update_W ->
convergence_diff -> batched subproblem solve), i.e. the body of
``PHBase.iterk_loop`` (mpisppy/phbase.py:901-970); the timed region is
``iterk_loop`` itself running K iterations (on the device: phx_iterk).  Workload: farmer,
crops_multiplier 1, 100,000 synthetic scenarios (configs[2] of BASELINE.json;
the metric is quoted on it and it fits one MI355X), rho = 1, scenarios sharded
contiguously over the ranks (strong scaling: the 100k total is fixed).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--scens S] [--cm C]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU)

Timed region: iterk_loop with PHIterLimit = K bracketed by barrier + device
synchronize; the MAX over ranks is reported.  Iter0 and W warmup iterations are
untimed.  --host-loop drives the iterations from Python instead.  Inputs are
resident in HBM before timing.  Extra keys:
  roofline      the dominant kernel of the timed region (the structure-
                specialised lane solver ``phx_lane_warm`` with the lane solver
                on, the PDHG chunk ``k_chunk`` otherwise): algorithmic bytes
                 / its average duration from HIP events recorded
                around it on the solve stream (every --timing-every-th iteration).
  cpu_baseline  the CPU restatement of the reference PH (oracle/cpu_bench.py:
                numpy + scipy-HiGHS + polish, one worker process per core) on a
                bounded sample, run as a child process on rank 0 at N = 1.
  conv_time     (--conv) wall time from Iter0 to conv < 1e-4.
"""
import argparse
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
    ap.add_argument("--scens", type=int, default=100000)
    ap.add_argument("--cm", type=int, default=1)
    ap.add_argument("--rho", type=float, default=1.0)
    ap.add_argument("--check-every", type=int, default=64)
    ap.add_argument("--ipm-after", type=int, default=None, help="PDHG iterations before the IPM finisher")
    ap.add_argument("--lane-solver", type=int, default=1, help="1: structure-specialised lane solver first")
    ap.add_argument("--as-rounds", type=int, default=None, help="active-set rounds (0: no warm active set)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-scens", type=int, default=40000)
    ap.add_argument("--cpu-iters", type=int, default=6)
    ap.add_argument("--cpu-procs", type=int, default=16, help="worker processes (the GPU box's CPU share)")
    ap.add_argument("--host-loop", action="store_true", help="drive each PH iteration from Python")
    ap.add_argument("--depth", type=int, default=4, help="phx_iterk: iterations kept enqueued ahead")
    ap.add_argument("--fused", type=int, default=1,
                    help="phx_iterk: one phx_lane_warm launch per PH iteration (Update_W + conv + solve + "
                         "next x-bar partials fused); 0: k_xbar, k_update_w_seg, warm, cold per iteration")
    ap.add_argument("--timing-every", type=int, default=5,
                    help="phx_iterk: HIP events around the lane kernel of every T-th iteration")
    ap.add_argument("--conv", action="store_true", help="also measure time to conv < 1e-4")
    ap.add_argument("--conv-max-iters", type=int, default=5000)
    return ap.parse_args()


def lane_bytes(b, fused=False):
    """Algorithmic HBM bytes of phx_lane_warm per scenario.

    reads : varying A values, W and rho of the nonant slots with their x-bar
            index (x-bar itself is a per-node vector, cache-resident), the
            active-set words, plus c / bounds / row bounds where they vary
    writes: x (n), row duals y (m), objective, status + iteration count
            (caller's and the context's), flags, active-set words
    The scenario-invariant data are literals of the JIT-specialised kernel.
    fused (phx_iterk fused mode): + the previous solve's nonant x and the
    prob_coeff (Update_W / next x-bar partials), + the W write-back.
    """
    nw = (2 * (b.n + b.m) + 31) // 32
    rd = 8 * (b.nvar + 2 * b.nonant.N) + 4 * b.nonant.N + 4 * nw
    rd += 8 * b.n * int(b.c_vary) + 16 * b.n * int(b.bnd_vary) + 16 * b.m * int(b.rhs_vary)
    wr = 8 * (b.n + b.m + 1) + 4 * 5 + 4 * nw
    if fused:
        rd += 16 * b.nonant.N
        wr += 8 * b.nonant.N
    return rd + wr


def pdhg_bytes(b):
    """Algorithmic bytes of one PDHG iteration of one scenario in k_chunk:
    the SpMM pair with de-duplicated A values
    8*(2*nnz_var + 2*n + 2*m) plus the fused vector updates 8*(7n + 5m)."""
    return 8 * (2 * b.nvar + 2 * b.n + 2 * b.m) + 8 * (7 * b.n + 5 * b.m)


def wg_bytes(b):
    """Algorithmic bytes of one scenario solve in k_wg_warm (phx_wg.h): reads
    the varying A values, qN/pN of the nonant slots and the warm-start point
    (x n, y m); writes x, x0, xT (3n) and y, y0, yT (3m) plus status + iters."""
    return 8 * (b.nvar + 2 * b.nonant.N + b.n + b.m) + 8 * (3 * b.n + 3 * b.m) + 8


def pmc_traffic(kernel, args):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC passes
    (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE; scripts/pmc_summary.py).
    Counters need their own profiler runs, so they are read from profiles/."""
    import glob
    if args.scens != 100000 or args.cm != 1:
        return None, None
    files = sorted(glob.glob(os.path.join(_ROOT, "profiles", "r*_pmc_%s.json" % kernel.replace("phx_", ""))))
    if not files:
        return None, None
    d = json.load(open(files[-1]))
    t = d.get("hbm_bytes_per_launch", {}).get("total")
    return t, os.path.relpath(files[-1], _ROOT)


def cpu_baseline(args):
    """oracle/cpu_bench.py in a child process (it never touches the GPU)."""
    procs = max(1, min(args.cpu_procs, os.cpu_count() or 1))
    cmd = [sys.executable, "-m", "oracle.cpu_bench", "--scens", str(args.cpu_scens), "--iters",
           str(args.cpu_iters), "--procs", str(procs), "--cm", str(args.cm), "--rho", str(args.rho)]
    r = subprocess.run(cmd, cwd=_ROOT, capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        return {"error": r.stderr[-500:]}
    d = json.loads(r.stdout.strip().splitlines()[-1])
    return {k: d[k] for k in ["value", "unit", "cores", "kind", "sample", "seconds"]}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local_rank)
        dist.init_process_group(backend="nccl")
    else:
        torch.cuda.set_device(0)
    import mpisppy_amd  # noqa: F401
    from mpisppy_amd.opt.ph import PH
    from mpisppy_amd.examples import farmer

    S = args.scens
    names = farmer.scenario_names_creator(S)
    solver_opts = {"pdhg_check_every": args.check_every, "lane_solver": args.lane_solver,
                   "iterk_depth": args.depth, "iterk_timing": args.timing_every, "iterk_fused": args.fused}
    if args.ipm_after is not None:
        solver_opts["ipm_after"] = args.ipm_after
    if args.as_rounds is not None:
        solver_opts["as_rounds"] = args.as_rounds
    opts = {"solver_name": "phx", "PHIterLimit": 10 ** 9, "defaultPHrho": args.rho, "convthresh": 1e-10,
            "verbose": False, "display_progress": False, "iter0_solver_options": dict(solver_opts),
            "iterk_solver_options": dict(solver_opts)}
    t_setup = time.perf_counter()
    ph = PH(opts, names, farmer.scenario_creator,
            scenario_creator_kwargs={"num_scens": S, "crops_multiplier": args.cm})
    ph.PH_Prep()
    ph.subproblem_creation(False)
    torch.cuda.synchronize()
    t_setup = time.perf_counter() - t_setup

    def step():
        ph._PHIter += 1
        ph.Compute_Xbar(False)
        ph.Update_W(False)
        ph.conv = ph.convergence_diff()
        ph.solve_loop(solver_options=ph.current_solver_options, gripe=False)

    t_iter0 = time.perf_counter()
    ph.Iter0()
    torch.cuda.synchronize()
    t_iter0 = time.perf_counter() - t_iter0
    K = args.steps
    b = ph.batch
    if args.host_loop or not ph._native_loop_ok():
        # one PHBase method call after the other from Python (the reference's loop body)
        for _ in range(args.warmup):
            step()
        ph._settle()
        n0 = len(ph.solve_stats)
        ph.mpicomm.Barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(K):
            step()
        ph._settle()             # the last solve may be deferred: finish it inside the timed region
        torch.cuda.synchronize()
        ph.mpicomm.Barrier()
        dt = time.perf_counter() - t0
        stats = ph.solve_stats[n0:]
        lane_warm_ms = sum(s.get("lane_warm_ms", 0.0) for s in stats)
        warm_launches = sum(1 for s in stats if s.get("lane_warm_ms", 0.0) > 0.0)
        loop_info = {"loop": "host (PHBase methods per iteration, deferred solves)"}
        fused_ran = False
    else:
        # PHBase.iterk_loop itself: with no per-iteration hooks it runs on the
        # device (phx_iterk: pipelined iterations, device-side stop test)
        ph.options["PHIterLimit"] = args.warmup
        ph.iterk_loop()
        torch.cuda.synchronize()
        ph.options["PHIterLimit"] = K
        ph.mpicomm.Barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ph.iterk_loop()
        torch.cuda.synchronize()
        ph.mpicomm.Barrier()
        dt = time.perf_counter() - t0
        st = getattr(ph, "iterk_stats", None)
        if st is None or st["iters"] != K or st["solves"] != K:
            raise RuntimeError("timed iterk_loop did not run %d full iterations: %s" % (K, st))
        stats = []
        lane_warm_ms = st["lane_warm_ms"]
        warm_launches = st["warm_launches"]
        fused_ran = bool(st.get("fused", False))
        loop_info = {"loop": "PHBase.iterk_loop -> phx_iterk (device-driven, depth %d%s)"
                             % (args.depth, ", fused: one launch per PH iteration" if fused_ran else ""),
                     "straggler_stops": st["straggler_stops"], "stragglers": st["stragglers"],
                     "not_optimal": st["not_optimal"]}
    dt_t = torch.tensor([dt], dtype=torch.float64, device="cuda")
    ph.mpicomm.allreduce_max_(dt_t)
    dt = float(dt_t.item())
    lane_on = lane_warm_ms > 0.0
    if lane_on:
        # dominant kernel: the warm active-set lane kernel, one launch per step over all local scenarios
        k_ms = lane_warm_ms
        launches = warm_launches
        bpu = lane_bytes(b, fused=fused_ran)
        units_per_launch = b.S
        kernel = "phx_lane_warm"
    elif sum(s.get("wg_ms", 0.0) for s in stats) > 0.0:
        # generic path with the workgroup warm active-set pass (medium subproblems)
        k_ms = sum(s.get("wg_ms", 0.0) for s in stats)
        launches = sum(1 for s in stats if s.get("wg_ms", 0.0) > 0.0)
        bpu = wg_bytes(b)
        units_per_launch = b.S
        kernel = "k_wg_warm"
    else:
        k_ms = sum(s["pdhg_ms"] for s in stats)
        launches = sum(s["launches"] for s in stats)
        bpu = pdhg_bytes(b)
        units_per_launch = sum(s["lane_iters"] for s in stats) / max(launches, 1)
        kernel = "k_chunk"
    avg_launch_s = k_ms / 1e3 / max(launches, 1)
    bytes_per_launch = bpu * units_per_launch
    achieved = bytes_per_launch / avg_launch_s / 1e9 if avg_launch_s > 0 else 0.0
    value = S * K / dt
    traffic, traffic_src = pmc_traffic(kernel, args) if world == 1 else (None, None)
    res = {
        "metric": "PH scenario-iterations/sec (farmer)",
        "value": value,
        "unit": "scenario-iterations/s",
        "n_gpus": world,
        "steps": K,
        "warmup": args.warmup,
        "ms_per_step": dt * 1e3 / K,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (farmer scenario generator, RandomState-seeded yields as the reference)",
        "config": {"workload": "farmer crops_multiplier=%d, %d scenarios, rho=%g, PH iterate" % (args.cm, S, args.rho),
                   "scenarios": S, "scenarios_per_gpu": b.S, "n": b.n, "m": b.m, "nnz": b.nnz,
                   "nnz_varying": b.nvar, "nonants": b.nonant.N,
                   "parallelism": "scenario-sharded x%d, RCCL allreduce" % world},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_unit": "bytes/launch",
                     "traffic_source": traffic_src, "algorithmic_bytes_per_launch": bytes_per_launch,
                     "kernel": kernel, "bytes_per_unit": bpu,
                     "unit_def": "scenario PDHG iteration" if kernel == "k_chunk" else "scenario solve",
                     "units_per_launch": units_per_launch,
                     "avg_launch_us": avg_launch_s * 1e6, "launches": launches},
        "loop": loop_info,
        # lane_warm: average sampled launch (one launch per step)
        "kernel_ms_per_step": {"lane_warm": lane_warm_ms / max(warm_launches, 1) if not stats else lane_warm_ms / K,
                               "lane_warm_list": sum(s.get("lane_warm_list_ms", 0.0) for s in stats) / K,
                               "lane_cold": sum(s.get("lane_ms", 0.0) for s in stats) / K,
                               "pdhg": sum(s["pdhg_ms"] for s in stats) / K,
                               "polish": sum(s["polish_ms"] for s in stats) / K,
                               "ipm": sum(s["ipm_ms"] for s in stats) / K,
                               "wg_warm": sum(s.get("wg_ms", 0.0) for s in stats) / K},
        "wg_certified_per_step": [s.get("wg_certified") for s in stats],
        "lane_certified_per_step": [s.get("lane_certified") for s in stats],
        "lane_warm_certified_per_step": [s.get("lane_warm_certified") for s in stats],
        "lane_first_certified_per_step": [s.get("lane_first_certified") for s in stats],
        "pdhg_iters_per_step": [s["pdhg_iters"] for s in stats],
        "solver_options": solver_opts,
        "not_optimal": sum(s["not_optimal"] for s in stats) if stats else loop_info.get("not_optimal"),
        "setup_s": t_setup, "iter0_s": t_iter0,
    }
    if args.conv:
        # time to conv < 1e-4 from Iter0 (fresh object, same data)
        del ph
        opts2 = dict(opts)
        opts2["convthresh"] = 1e-4
        opts2["PHIterLimit"] = args.conv_max_iters
        ph2 = PH(opts2, names, farmer.scenario_creator,
                 scenario_creator_kwargs={"num_scens": S, "crops_multiplier": args.cm})
        torch.cuda.synchronize()
        ph2.mpicomm.Barrier()
        t0 = time.perf_counter()
        ph2.ph_main(finalize=False)
        torch.cuda.synchronize()
        tc = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device="cuda")
        ph2.mpicomm.allreduce_max_(tc)
        res["conv_time"] = {"seconds": float(tc.item()), "iterations": ph2._PHIter,
                            "conv": ph2.conv, "convthresh": 1e-4}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(args)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
