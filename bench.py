"""bench.py — PH scenario-iterations/s on farmer (BASELINE.json metric).

A "step" is one PH iteration over every scenario (Compute_Xbar -> Update_W ->
convergence_diff -> batched subproblem solve), i.e. the body of
``PHBase.iterk_loop`` (mpisppy/phbase.py:901-970).  Workload: farmer,
crops_multiplier 1, 100,000 synthetic scenarios (configs[2] of BASELINE.json;
the metric is quoted on it and it fits one MI355X), rho = 1, scenarios sharded
contiguously over the ranks (strong scaling: total scenarios fixed).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--scens S] [--cm C]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU)

Timed region: K steps bracketed by barrier + device synchronize; the MAX over
ranks is reported.  Iter0 and W warmup steps are untimed.  Inputs are resident
in HBM before timing.  Extra keys: roofline (dominant kernel k_chunk, HIP
event timing, algorithmic bytes per DESIGN.md §4), cpu_baseline (the CPU
oracle — numpy + scipy HiGHS — on a bounded sample, rank 0, N=1 only),
conv_time (time to conv < 1e-4 when --conv is given).
"""
import argparse
import json
import os
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
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--scens", type=int, default=100000)
    ap.add_argument("--cm", type=int, default=1)
    ap.add_argument("--rho", type=float, default=1.0)
    ap.add_argument("--check-every", type=int, default=64)
    ap.add_argument("--ipm-after", type=int, default=None, help="PDHG iterations before the IPM finisher")
    ap.add_argument("--lane-solver", type=int, default=1, help="1: structure-specialised lane IPM first")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=400)
    ap.add_argument("--conv", action="store_true", help="also measure time to conv < 1e-4")
    ap.add_argument("--conv-max-iters", type=int, default=3000)
    return ap.parse_args()


def bytes_per_lane_iter(b):
    """Algorithmic bytes of one PDHG iteration of one scenario in k_chunk.

    SpMM pair with de-duplicated A values:
        8 * (2*nnz_var + 2*n + 2*m)
    plus the fused vector updates of the iteration:  8 * (7*n + 5*m).
    """
    return 8 * (2 * b.nvar + 2 * b.n + 2 * b.m) + 8 * (7 * b.n + 5 * b.m)


def cpu_baseline(args):
    """The CPU oracle (HiGHS + KKT polish, numpy PH) on a bounded sample."""
    from oracle import models as om, ph as oph
    S = args.cpu_sample
    scens = [om.farmer("scen%d" % i, crops_multiplier=args.cm, num_scens=S) for i in range(S)]
    o = oph.OraclePH(scens, rho=args.rho)
    o.iter0()
    K = 2
    t0 = time.perf_counter()
    for _ in range(K):
        o.compute_xbar()
        o.update_w()
        o.convergence_diff()
        o.solve_loop()
    dt = time.perf_counter() - t0
    return {"value": S * K / dt, "unit": "scenario-iterations/s", "cores": 1, "kind": "port",
            "sample": "oracle PH (numpy + scipy-HiGHS 1.8 QP + KKT polish), farmer cm=%d, %d scenarios x %d "
                      "PH iterations after Iter0, 1 core" % (args.cm, S, K)}


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
    solver_opts = {"pdhg_check_every": args.check_every, "lane_solver": args.lane_solver}
    if args.ipm_after is not None:
        solver_opts["ipm_after"] = args.ipm_after
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
    for _ in range(args.warmup):
        step()
    n0 = len(ph.solve_stats)
    ph.mpicomm.Barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    ph.mpicomm.Barrier()
    dt = time.perf_counter() - t0
    dt_t = torch.tensor([dt], dtype=torch.float64, device="cuda")
    ph.mpicomm.allreduce_max_(dt_t)
    dt = float(dt_t.item())
    stats = ph.solve_stats[n0:]
    pdhg_ms = sum(s["pdhg_ms"] for s in stats)
    launches = sum(s["launches"] for s in stats)
    lane_iters = sum(s["lane_iters"] for s in stats)
    b = ph.batch
    bpl = bytes_per_lane_iter(b)
    avg_launch_s = pdhg_ms / 1e3 / max(launches, 1)
    bytes_per_launch = lane_iters * bpl / max(launches, 1)
    achieved = bytes_per_launch / avg_launch_s / 1e9 if avg_launch_s > 0 else 0.0
    value = S * args.steps / dt
    res = {
        "metric": "PH scenario-iterations/sec (farmer)",
        "value": value,
        "unit": "scenario-iterations/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (farmer scenario generator, RandomState-seeded yields as the reference)",
        "config": {"workload": "farmer crops_multiplier=%d, %d scenarios, rho=%g, PH iterate" % (args.cm, S, args.rho),
                   "scenarios": S, "scenarios_per_gpu": b.S, "n": b.n, "m": b.m, "nnz": b.nnz,
                   "nnz_varying": b.nvar, "parallelism": "scenario-sharded x%d, RCCL allreduce" % world},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                     "kernel": "k_chunk", "bytes_per_scenario_iter": bpl,
                     "avg_launch_us": avg_launch_s * 1e6, "launches": launches,
                     "scenario_iters_per_launch": lane_iters / max(launches, 1)},
        "pdhg_iters_per_step": [s["pdhg_iters"] for s in stats],
        "kernel_ms_per_step": {"pdhg": pdhg_ms / args.steps, "polish": sum(s["polish_ms"] for s in stats) / args.steps,
                               "ipm": sum(s["ipm_ms"] for s in stats) / args.steps,
                               "lane_ipm": sum(s.get("lane_ms", 0.0) for s in stats) / args.steps,
                               "lane_warm": sum(s.get("lane_warm_ms", 0.0) for s in stats) / args.steps},
        "lane_certified_per_step": [s.get("lane_certified") for s in stats],
        "lane_warm_certified_per_step": [s.get("lane_warm_certified") for s in stats],
        "solver_options": solver_opts,
        "not_optimal": sum(s["not_optimal"] for s in stats),
        "setup_s": t_setup, "iter0_s": t_iter0,
    }
    if args.conv:
        # time to conv < 1e-4 from Iter0 (fresh object)
        del ph
        opts2 = dict(opts)
        opts2["convthresh"] = 1e-4
        opts2["PHIterLimit"] = args.conv_max_iters
        ph2 = PH(opts2, names, farmer.scenario_creator,
                 scenario_creator_kwargs={"num_scens": S, "crops_multiplier": args.cm})
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ph2.ph_main(finalize=False)
        torch.cuda.synchronize()
        res["conv_time"] = {"seconds": time.perf_counter() - t0, "iterations": ph2._PHIter,
                            "conv": ph2.conv, "convthresh": 1e-4}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(args)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
