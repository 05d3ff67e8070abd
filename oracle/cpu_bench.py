"""CPU baseline for bench.py — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

The reference's PH iterate as it runs under ``mpiexec -n P`` (one process per
core, contiguous scenario slices ``range(int(r*S/P), int((r+1)*S/P))``,
``utils/sputils.py:803-810``), restated with the oracle: each worker process
owns its slice and solves its subproblems with scipy-HiGHS + KKT polish
(``SPOpt.solve_loop``, ``spopt.py:226-307``); the parent plays the per-node
Allreduce of ``_Compute_Xbar`` (``phbase.py:83-87``).  No Pyomo model layer, so
this is FASTER than the reference itself: a conservative baseline.

Timed: K PH iterations (Compute_Xbar -> Update_W -> convergence_diff ->
solve_loop) after an untimed Iter0.  Prints one JSON line.

    python -m oracle.cpu_bench --scens 4000 --iters 3 --procs 16

Run by bench.py as a CHILD PROCESS (it never touches the GPU).
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)

from oracle import models as om, ph as oph  # noqa: E402


AIRCOND_BF = [10, 10, 10]       # C4 (BASELINE configs[3])


def make_scen(model, nm, S, cm=1):
    """One oracle scenario of the bench workloads (two-stage: one ROOT x-bar;
    aircond: the multistage tree of C4, x-bar per tree node)."""
    if model == "aircond":
        return om.aircond(nm, AIRCOND_BF)
    if model == "farmer":
        return om.farmer(nm, crops_multiplier=cm, num_scens=S)
    if model == "sslp":
        return om.sslp(nm, num_scens=S)
    if model == "netdes50":
        return om.netdes(nm, "network-50-30-H-01", num_scens=S)
    raise ValueError(model)


def names_of(model, S):
    if model in ("farmer", "aircond"):
        return ["scen%d" % i for i in range(S)]
    if model == "sslp":
        return ["Scenario%d" % (i + 1) for i in range(S)]
    return ["Scenario%d" % i for i in range(S)]


def fast_solver(scens):
    """The baseline's per-subproblem solve: a persistent HiGHS instance per scenario
    (costs and prox Hessian changed per solve, warm from its last basis: the
    reference's persistent solver plugins) + one dense KKT polish of its basis
    (qp.solve_fast; the iterated certified polish only when that point fails the
    certificate) for small subproblems; the oracle's sparse path (qp.solve) for large
    ones (sslp, netdes)."""
    from oracle import qp
    small = all(s.A.shape[0] + s.A.shape[1] <= 300 for s in scens)
    if not small:
        return qp.solve
    inst = {id(s.A): qp.PersistentHighs(s.A, s.bl, s.bu, s.lb, s.ub) for s in scens}

    def solve(A, bl, bu, lb, ub, q, p):
        return qp.solve_fast(A, bl, bu, lb, ub, q, p, hs=inst.get(id(A)))
    return solve


def _node_partials(o):
    """The worker's share of _Compute_Xbar's per-node sums (phbase.py:54-80):
    {(node, slot): [sum pc x, sum pc x^2]} over its scenarios (multistage)."""
    xn = o.xn()
    part = {}
    for k in range(o.S):
        for j in range(o.N):
            a = part.setdefault((o.node_of[k][j], j), [0.0, 0.0])
            v = o.pc[k, j] * xn[k, j]
            a[0] += v
            a[1] += v * xn[k, j]
    return part


def _worker(conn, names, S, cm, rho, model="farmer"):
    scens = [make_scen(model, nm, S, cm) for nm in names]
    o = oph.OraclePH(scens, rho=rho)
    o.solver = fast_solver(scens)
    o.iter0()
    multi = model == "aircond"
    conn.send((_node_partials(o) if multi else o.xn(), o.obj.copy()))
    while True:
        msg = conn.recv()
        if msg is None:
            break
        if multi:      # the all-reduced node sums: x-bar per (node, slot)
            for k in range(o.S):
                for j in range(o.N):
                    o.xbar[k, j] = msg[(o.node_of[k][j], j)]
        else:
            o.xbar[:] = msg[None, :]
        o.update_w()
        d = float(np.sum(np.abs(o.xn() - o.xbar)))
        o.solve_loop()
        conn.send((_node_partials(o) if multi else o.xn(), d))
    conn.close()


def run(S, K, P, cm=1, rho=1.0, model="farmer", S_total=None):
    """K PH iterations over a sample of S scenarios (probabilities 1/S_total: the
    subproblems of the full workload; x-bar over the sample)."""
    St = S_total or S
    names = names_of(model, S)
    avg = S / P
    slices = [names[int(r * avg):int((r + 1) * avg)] for r in range(P)]
    ctx = mp.get_context("fork")
    pipes, procs = [], []
    t_setup = time.perf_counter()
    for sl in slices:
        a, b = ctx.Pipe()
        p = ctx.Process(target=_worker, args=(b, sl, St, cm, rho, model))
        p.start()
        pipes.append(a)
        procs.append(p)
    res = [c.recv() for c in pipes]          # Iter0 done everywhere
    t_setup = time.perf_counter() - t_setup
    multi = model == "aircond"
    prob = 1.0 / S                           # x-bar over the sample
    t0 = time.perf_counter()
    conv = None
    for _ in range(K):
        if multi:
            # the per-node Allreduce (phbase.py:83-87): the full tree is run
            tot = {}
            for r in res:
                for key, (a, b) in r[0].items():
                    t = tot.setdefault(key, [0.0, 0.0])
                    t[0] += a
                    t[1] += b
            xbar = {key: v[0] for key, v in tot.items()}
            nslot = 1 + max(j for (_, j) in tot)
        else:
            xn = np.concatenate([r[0] for r in res])
            xbar = prob * xn.sum(axis=0)     # Compute_Xbar (+ the Allreduce)
            nslot = xn.shape[1]
        for c in pipes:
            c.send(xbar)
        res = [c.recv() for c in pipes]
        conv = sum(r[1] for r in res) / (S * nslot)
    dt = time.perf_counter() - t0
    for c in pipes:
        c.send(None)
    for p in procs:
        p.join()
    return {"value": S * K / dt, "unit": "scenario-iterations/s", "cores": P, "kind": "port",
            "seconds": dt, "setup_and_iter0_seconds": t_setup, "conv_last": conv,
            "sample": "oracle PH restatement (numpy + persistent scipy-HiGHS 1.8 LP/QP + one KKT polish of its basis; "
                      "sparse IPM + certified polish above 300 rows+cols), %s, %d scenarios x %d PH iterations "
                      "after Iter0, %d worker processes (contiguous slices, parent = Allreduce)"
                      % ("farmer cm=%d" % cm if model == "farmer" else
                         ("aircond %s (the whole tree, per-node x-bar)" % "x".join(map(str, AIRCOND_BF))
                          if model == "aircond" else model), S, K, P),
            "host": host_info()}


def host_info():
    """nproc, physical cores / sockets (distinct (physical id, core id) pairs of
    /proc/cpuinfo: lscpu's cores x sockets) and the CPU model of the machine
    the baseline ran on."""
    model = None
    cores, sockets, phys, core = set(), set(), None, None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                k, _, v = line.partition(":")
                k, v = k.strip(), v.strip()
                if k == "model name" and model is None:
                    model = v
                elif k == "physical id":
                    phys = v
                    sockets.add(v)
                elif k == "core id":
                    core = v
                elif not k:
                    if phys is not None and core is not None:
                        cores.add((phys, core))
                    phys = core = None
        if phys is not None and core is not None:
            cores.add((phys, core))
    except OSError:
        pass
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None
    return {"nproc": os.cpu_count(), "affinity_cpus": aff, "cpu_model": model,
            "physical_cores": len(cores) or None, "sockets": len(sockets) or None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scens", type=int, default=4000)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--procs", type=int, default=min(16, os.cpu_count() or 1))
    ap.add_argument("--cm", type=int, default=1)
    ap.add_argument("--rho", type=float, default=1.0)
    ap.add_argument("--model", default="farmer", choices=["farmer", "sslp", "netdes50", "aircond"])
    ap.add_argument("--scens-total", type=int, default=None, help="probability 1/S_total (the full workload)")
    a = ap.parse_args()
    print(json.dumps(run(a.scens, a.iters, a.procs, a.cm, a.rho, a.model, a.scens_total)), flush=True)


if __name__ == "__main__":
    main()
