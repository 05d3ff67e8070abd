"""Scenario-tree node attached to each scenario model.

Mirrors ``mpisppy.scenario_tree.ScenarioNode`` (``mpisppy/scenario_tree.py:44-96``):
same constructor, same ``nonant_vardata_list`` expansion rule
(``build_vardatalist``, sorted keys for indexed variables).
"""
import logging

from .model import build_vardatalist

logger = logging.getLogger("mpisppy_amd.scenario_tree")


class ScenarioNode:
    def __init__(self, name, cond_prob, stage, cost_expression, nonant_list, scen_model,
                 nonant_ef_suppl_list=None, parent_name=None):
        self.name = name
        self.cond_prob = cond_prob
        self.stage = stage
        self.cost_expression = cost_expression
        self.nonant_list = nonant_list
        self.nonant_ef_suppl_list = nonant_ef_suppl_list
        self.parent_name = parent_name
        if nonant_list is not None:
            self.nonant_vardata_list = build_vardatalist(nonant_list)
        else:
            logger.warning("nonant_list is empty for node %s, no nonanticipativity "
                           "will be enforced at this node by default", name)
            self.nonant_vardata_list = []
        if nonant_ef_suppl_list is not None:
            self.nonant_ef_suppl_vardata_list = build_vardatalist(nonant_ef_suppl_list)
        else:
            self.nonant_ef_suppl_vardata_list = []
