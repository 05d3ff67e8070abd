"""Lane-solver statistics from the host emulation (no GPU): builds the emu
library with extra -D flags (a variant under /tmp), runs farmer PH for a few
iterations with PHX_EMU_DEBUG=1 and summarises, per solve, the wave-max rounds
(a 64-lane wavefront runs as long as its slowest lane), rounds and refinement
steps per lane.
    python scripts/emu_stats.py [S] [iters] [-DNAME=VAL ...]"""
import os
import re
import subprocess
import sys

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def build(flags):
    tag = "_".join(f.lstrip("-D").replace("=", "") for f in flags) or "base"
    out = "/tmp/emu_%s.so" % tag
    src = os.path.join(_ROOT, "tests", "emu", "phx_emu.cpp")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-fPIC", "-shared"] + flags + ["-o", out, src])
    return out


CHILD = r'''
import os, sys
sys.path.insert(0, %(root)r); sys.path.insert(0, os.path.join(%(root)r, "tests"))
import mpisppy_amd
from mpisppy_amd import _native
from mpisppy_amd.examples import farmer
from helpers import ph_options
from mpisppy_amd.opt.ph import PH
lib = _native.Lib(%(so)r, prefix="emu_phx_")
S, K = %(S)d, %(K)d
opts = ph_options(K)
opts["iterk_solver_options"] = dict({"native_loop": 0}, **dict(%(sok)s))
opts["iter0_solver_options"] = dict(%(so0)s)
ph = PH(opts, farmer.scenario_names_creator(S), farmer.scenario_creator, scenario_creator_kwargs={"num_scens": S},
        _native_lib=lib, _device="cpu")
conv, E, tb = ph.ph_main()
print("RESULT", conv, E, tb)
'''


def main():
    a = sys.argv[1:]
    flags = [x for x in a if x.startswith("-D")]
    pos = [x for x in a if not x.startswith("-D")]
    S = int(pos[0]) if pos else 2000
    K = int(pos[1]) if len(pos) > 1 else 10
    so = build(flags)
    env = dict(os.environ, PHX_EMU_DEBUG="1")
    so0 = os.environ.get("EMU_SO0", "{}")
    sok = os.environ.get("EMU_SOK", "{}")      # iterk solver options (e.g. as_rounds)
    r = subprocess.run([sys.executable, "-c", CHILD % {"root": _ROOT, "so": so, "S": S, "K": K, "so0": so0, "sok": sok}],
                       capture_output=True, text=True, env=env)
    k = 0
    for line in r.stderr.splitlines():
        m = re.match(r"\[emu first pass\] wave-max rounds ([\d.]+) \|(.*)", line)
        if m:
            print("solve %2d  wave-max rounds %s  hist %s" % (k, m.group(1), m.group(2).strip()[:80]))
        m = re.match(r"\[emu lane stats\] rounds=(\d+) refine=(\d+)", line)
        if m:
            ro, rf = int(m.group(1)), int(m.group(2))
            print("solve %2d  rounds/lane %.3f  refine/round %.3f" % (k, ro / S, rf / max(ro, 1)))
            k += 1
        if line.startswith("[emu rescue") or line.startswith("[emu cold"):
            print("          " + line[:120])
    # -DPHX_EMU_REFINE_TRACE: per refinement solve, the sequence of relative corrections
    seqs, cur = [], []
    for line in r.stderr.splitlines():
        if line.startswith("[refine]"):
            st, v = line.split()[1:]
            if int(st) == 0 and cur:
                seqs.append(cur)
                cur = []
            cur.append(float(v))
    if cur:
        seqs.append(cur)
    if seqs:
        import collections
        tail = seqs[-min(len(seqs), 20000):]
        lens = collections.Counter(len(q) for q in tail)
        print("refinement solves %d (last %d): steps %s" % (len(seqs), len(tail), sorted(lens.items())))
        for L in sorted(lens):
            sel = [q for q in tail if len(q) == L]
            mean = [sum(q[k] for q in sel) / len(sel) for k in range(L)]
            print("  %d steps (%d): mean log10 rel. correction per step %s" % (L, len(sel), " ".join("%.1f" % v for v in mean)))
    for line in r.stdout.splitlines():
        if line.startswith("RESULT"):
            print(line)
    if r.returncode:
        print(r.stderr[-2000:])


if __name__ == "__main__":
    main()
