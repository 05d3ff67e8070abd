"""Scenario-tree utilities used on the PH path.

Restatements of the reference helpers in ``mpisppy/utils/sputils.py``:
``extract_num`` (481-490), ``node_idx`` (492-519), ``parent_ndn`` (544-548),
``create_nodenames_from_branching_factors`` (934-959), ``attach_root_node``
(844-860) and the contiguous rank-slicing rule of
``_ScenTree.scen_names_to_ranks`` (774-840, slices at 803-810).
"""
import re

import numpy as np

from ..scenario_tree import ScenarioNode


def extract_num(string):
    return int(re.compile(r"(\d+)$").search(string).group(1))


def _nodenum_before_stage(t, branching_factors):
    return int(sum(np.prod(branching_factors[0:i]) for i in range(t)))


def node_idx(node_path, branching_factors):
    if node_path == []:
        return 0
    stage_id = 0
    for t in range(len(node_path)):
        stage_id = node_path[t] + branching_factors[t] * stage_id
    return _nodenum_before_stage(len(node_path), branching_factors) + stage_id


def parent_ndn(nodename):
    if nodename == "ROOT":
        return None
    return re.search(r"(.+)_(\d+)", nodename).group(1)


def create_nodenames_from_branching_factors(BFS):
    stage_nodes = ["ROOT"]
    nodenames = ["ROOT"]
    if len(BFS) == 1:
        return nodenames
    for bf in BFS:
        old = stage_nodes
        stage_nodes = []
        for k in range(len(old)):
            stage_nodes += ["%s_%i" % (old[k], b) for b in range(bf)]
        nodenames += stage_nodes
    return nodenames


def rank_slices(scen_count, n_proc):
    """rank -> list of scenario indices; contiguous, ``int(r*S/R)`` boundaries."""
    if n_proc == 1:
        return [list(range(scen_count))]
    avg = scen_count / n_proc
    return [list(range(int(i * avg), int((i + 1) * avg))) for i in range(n_proc)]


def rank_bounds(scen_count, n_proc):
    """[(first, last+1)] per rank, same rule as :func:`rank_slices`."""
    if n_proc == 1:
        return [(0, scen_count)]
    avg = scen_count / n_proc
    return [(int(i * avg), int((i + 1) * avg)) for i in range(n_proc)]


def attach_root_node(model, firstobj, varlist, nonant_ef_suppl_list=None):
    model._mpisppy_node_list = [
        ScenarioNode("ROOT", 1.0, 1, firstobj, varlist, model,
                     nonant_ef_suppl_list=nonant_ef_suppl_list)
    ]


def find_leaves(all_nodenames):
    if all_nodenames is None or all_nodenames == ["ROOT"]:
        return {"ROOT": False}
    s = set(all_nodenames)
    return {ndn: (ndn + "_0") not in s for ndn in all_nodenames}
