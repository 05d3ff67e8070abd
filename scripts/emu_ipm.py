"""Iter0 interior-point iterations per lane in the host emulation (no GPU),
for an emu variant built with extra -D flags: farmer S scenarios, unseeded
(every lane cold).  python scripts/emu_ipm.py [S] [-DNAME=VAL ...]"""
import collections
import os
import subprocess
import sys

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(_ROOT, "scripts"))
from emu_stats import build  # noqa: E402

CHILD = r'''
import os, sys, collections
sys.path.insert(0, %(root)r); sys.path.insert(0, os.path.join(%(root)r, "tests"))
import mpisppy_amd
from mpisppy_amd import _native
from mpisppy_amd.examples import farmer, aircond, hydro
from mpisppy_amd.utils import sputils
from helpers import ph_options
from mpisppy_amd.opt.ph import PH
lib = _native.Lib(%(so)r, prefix="emu_phx_")
S = %(S)d
opts = ph_options(0)
opts["iter0_solver_options"] = {"seed_templates": 0}
if %(model)r == "farmer":
    names, cr, kw, nodes = farmer.scenario_names_creator(S), farmer.scenario_creator, {"num_scens": S}, None
else:
    bfs = [10, 10, max(1, S // 100)]
    S = 100 * bfs[2]
    names, cr, kw = ["scen%%d" %% i for i in range(S)], aircond.scenario_creator, {"branching_factors": bfs}
    nodes = sputils.create_nodenames_from_branching_factors(bfs)
ph = PH(opts, names, cr, scenario_creator_kwargs=kw, all_nodenames=nodes, _native_lib=lib, _device="cpu")
ph.PH_Prep(); ph.subproblem_creation(False); ph._defer_iter0_checks = False; ph.Iter0()
it = ph._iters.numpy().tolist()
w = [max(it[k:k + 64]) for k in range(0, S, 64)]
print("IPM its", sorted(collections.Counter(it).items()), "mean %%.2f wave-max mean %%.2f" %% (sum(it) / S, sum(w) / len(w)),
      "not_optimal", ph.solve_stats[-1]["not_optimal"], "tb %%.12g" %% ph.trivial_bound)
'''


def main():
    a = sys.argv[1:]
    flags = [x for x in a if x.startswith("-D")]
    pos = [x for x in a if not x.startswith("-D")]
    S = int(pos[0]) if pos else 2000
    so = build(flags)
    model = os.environ.get("EMU_MODEL", "farmer")
    r = subprocess.run([sys.executable, "-c", CHILD % {"root": _ROOT, "so": so, "S": S, "model": model}],
                       capture_output=True, text=True)
    print(" ".join(flags) or "base", r.stdout.strip() or r.stderr[-1500:])


if __name__ == "__main__":
    main()
