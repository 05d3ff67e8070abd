"""Run one engine case on the GPU outside pytest (debugging aid)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import mpisppy_amd  # noqa
from helpers import run_engine  # noqa
from mpisppy_amd.examples import aircond  # noqa
from mpisppy_amd.utils import sputils  # noqa

bfs = [3, 3, 2]
nl = int(os.environ.get("NL", "0"))
opts = {"iter0_solver_options": {}, "iterk_solver_options": {"native_loop": nl}}
r = run_engine(aircond.scenario_creator, ["scen%d" % i for i in range(18)], {"branching_factors": bfs, "start_seed": 0},
               5, all_nodenames=sputils.create_nodenames_from_branching_factors(bfs), options=opts)
print("ok", r[1:])
