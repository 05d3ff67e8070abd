"""W and x-bar CSV checkpoint I/O (mpisppy/utils/wxbarutils.py:42-395).

File formats (identical to the reference's, so files move between the two):

* W, one main file:      ``scenario_name,variable_name,value`` per row
  (``write_W_to_file`` :42-84 appends; rows in local-scenario, nonant order);
* W, one file per scenario (``sep_files``): ``<dir>/<sname>_weights.csv`` with
  ``variable_name,value`` rows;
* x-bar:                 ``variable_name,value`` per nonant of the first local
  scenario (``write_xbar_to_file`` :280-301, rank 0, append mode).

Rows starting with ``#`` are comments; variable names may contain commas (the
value is the last field, the scenario name the first).  Values are written with
``str(float)`` (shortest round-trip repr), as the reference does.

The state lives on the device: W is read/written in bulk as the ``[N][S]``
tensor (one transfer, not one per element), x-bar through the per-node buffer
every scenario's slots index (``_xbar_idx``).  Error behaviour follows the
reference: missing scenarios / variables raise ``RuntimeError`` (:226-229,
:248-252, :339-341), unknown ones are reported and ignored, and W files must be
dual feasible, sum_s p_s W_s = 0 within 1e-7 (:262-277).
"""
import os

import numpy as np
import torch


def _slot_names(PHB):
    """nonant variable name of every slot, in slot order (same for every scenario)."""
    nn = PHB.batch.nonant
    return [nn.var_names[j] for j in range(nn.N)]


def _local_names(PHB):
    return list(PHB.local_scenarios.keys())


# ----------------------------------------------------------------------- W
def write_W_to_file(PHB, fname, sep_files=False):
    """Write every local scenario's W (wxbarutils.py:42-84); the main-file form
    gathers all ranks' rows to rank 0, which appends them in rank order."""
    names = _slot_names(PHB)
    W = PHB.W_array()                     # (S_local, N)
    snames = _local_names(PHB)
    if sep_files:
        os.makedirs(fname, exist_ok=True)
        for s, sname in enumerate(snames):
            with open(os.path.join(fname, sname + "_weights.csv"), "w") as f:
                for j, vn in enumerate(names):
                    f.write("%s,%s\n" % (vn, str(float(W[s, j]))))
        return
    rows = ["%s,%s,%s\n" % (sname, vn, str(float(W[s, j])))
            for s, sname in enumerate(snames) for j, vn in enumerate(names)]
    allrows = PHB.comms["ROOT"].gather(rows, root=0)
    if PHB.cylinder_rank == 0:
        with open(fname, "a") as f:
            for part in allrows:
                f.writelines(part)


def _parse_W_csv_single(fname):
    """{variable_name: value} from one scenario's W file (:131-153)."""
    if not os.path.exists(fname):
        raise RuntimeError("Could not find file {fn}".format(fn=fname))
    out = {}
    with open(fname) as f:
        for line in f:
            if line.startswith("#"):
                continue
            parts = line.rstrip("\n").split(",")
            out[",".join(parts[:-1])] = float(parts[-1])
    return out


def _parse_W_csv(fname, scenario_names_local, scenario_names_global, rank):
    """{scenario: {variable: value}} for the local scenarios from a main W file
    (:156-229): unknown scenarios are reported (rank 0) and skipped, a missing
    local scenario raises RuntimeError."""
    known = set(scenario_names_global)
    local = set(scenario_names_local)
    out = {}
    with open(fname) as f:
        for line in f:
            if line.startswith("#"):
                continue
            parts = line.rstrip("\n").split(",")
            sname, vname, val = parts[0], ",".join(parts[1:-1]), float(parts[-1])
            if sname not in known:
                if rank == 0:
                    print("WARNING: Ignoring unknown scenario name", sname)
                continue
            if sname in local:
                out.setdefault(sname, {})[vname] = val
    missing = [s for s in scenario_names_local if s not in out]
    if missing:
        raise RuntimeError("rank " + str(rank) + " could not find the following "
                           "scenarios in the provided weight file: " + ", ".join(missing))
    return out


def _check_W(w_val_dict, PHB, rank):
    """Missing variables raise, extra ones are dropped with a message, and the
    weights must satisfy sum_s p_s W_s = 0 per variable (:232-277)."""
    want = set(_slot_names(PHB))
    for sname in _local_names(PHB):
        have = set(w_val_dict[sname].keys())
        miss = want - have
        if miss:
            raise RuntimeError(sname + " is missing the following variables: " + ", ".join(sorted(miss)))
        extra = have - want
        if extra:
            print("Removing unknown variables:", ", ".join(sorted(extra)))
            for v in extra:
                w_val_dict[sname].pop(v, None)
    prob = {s: PHB.local_scenarios[s]._mpisppy_probability for s in _local_names(PHB)}
    local = {v: sum(prob[s] * w_val_dict[s][v] for s in _local_names(PHB)) for v in want}
    parts = PHB.comms["ROOT"].gather(local, root=0)
    if rank == 0:
        for v in sorted(want):
            if abs(sum(p[v] for p in parts)) > 1e-7:
                raise RuntimeError("Provided weights do not satisfy dual feasibility: "
                                   "\\sum_{scenarios} prob(s) * w(s) != 0. Error on variable " + v)


def set_W_from_file(fname, PHB, rank, sep_files=False, disable_check=False):
    """Load W for every local scenario (:87-128) into the device tensor."""
    snames = _local_names(PHB)
    if sep_files:
        vals = {s: _parse_W_csv_single(os.path.join(fname, s + "_weights.csv")) for s in snames}
    else:
        vals = _parse_W_csv(fname, snames, PHB.all_scenario_names, rank)
    if not disable_check:
        _check_W(vals, PHB, rank)
    names = _slot_names(PHB)
    N, S = len(names), len(snames)
    W = PHB._host("W").copy()            # (N, S_local): keeps slots a file leaves out (disable_check)
    for s, sname in enumerate(snames):
        d = vals[sname]
        for j, vn in enumerate(names):
            if vn in d:
                W[j, s] = d[vn]
    if N:
        PHB._W.copy_(torch.from_numpy(np.ascontiguousarray(W).reshape(-1)).to(PHB._W.device))
    PHB._bump()


# -------------------------------------------------------------------- x-bar
def write_xbar_to_file(PHB, fname):
    """Append the first local scenario's x-bars, rank 0 only (:280-301)."""
    if PHB.cylinder_rank != 0:
        return
    xb = PHB._host("xbar")
    idx = PHB._xbar_idx[:, 0]
    with open(fname, "a") as f:
        for j, vn in enumerate(_slot_names(PHB)):
            f.write("%s,%s\n" % (vn, str(float(xb[int(idx[j])]))))


def _parse_xbar_csv(fname):
    """{variable_name: value} (:327-361)."""
    out = {}
    with open(fname) as f:
        for line in f:
            if line.startswith("#"):
                continue
            parts = line.rstrip("\n").split(",")
            out[",".join(parts[:-1])] = float(parts[-1])
    return out


def _check_xbar(xbar_val_dict, PHB):
    """Every nonant needs a value (RuntimeError); extras are reported (:364-381)."""
    want = set(_slot_names(PHB))
    have = set(xbar_val_dict.keys())
    miss = want - have
    if miss:
        raise RuntimeError("Could not find the following required variable values in the provided "
                           "input file: " + ", ".join(sorted(miss)))
    extra = have - want
    if extra:
        print("Ignoring the following variables values provided in the input file: " + ", ".join(sorted(extra)))


def set_xbar_from_file(fname, PHB):
    """x-bar (and xsqbar = x-bar^2) of every node a local scenario touches, by
    variable name (:304-324)."""
    vals = _parse_xbar_csv(fname)
    if PHB.cylinder_rank == 0:
        _check_xbar(vals, PHB)
    names = _slot_names(PHB)
    xb = PHB._host("xbar").copy()
    xs = PHB._host("xsqbar").copy()
    idx = np.asarray(PHB._xbar_idx)
    for j, vn in enumerate(names):
        v = vals[vn]
        for i in np.unique(idx[j]):
            xb[int(i)] = v
            xs[int(i)] = v * v
    PHB._xbar_node.copy_(torch.from_numpy(xb).to(PHB._xbar_node.device))
    PHB._xsqbar_node.copy_(torch.from_numpy(xs).to(PHB._xsqbar_node.device))
    PHB._bump()


def ROOT_xbar_npy_serializer(PHB, fname):
    """ROOT-node x-bar as a numpy text file (:384-395)."""
    np.savetxt(fname, PHB.xbar_by_node()["ROOT"][0])
