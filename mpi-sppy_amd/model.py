"""Lightweight linear scenario models (the data a ``scenario_creator`` returns).

The reference's scenario creators return Pyomo ``ConcreteModel`` objects
carrying ``_mpisppy_node_list`` and ``_mpisppy_probability``
(``mpisppy/spbase.py:255-291, 505-522``).  Pyomo is not part of this stack, so
scenario creators written for this engine build a :class:`LinearModel`
instead: named variables with bounds, linear rows ``lb <= a'x <= ub``, a linear
objective and the same scenario-tree attachments.  The engine only ever needs
the model's standard form (``LinearModel.standard_form``); everything else the
reference reads from Pyomo objects (W, xbars, rho, nonant values) is exposed by
the engine through views (see ``spbase.ScenarioView``).

Nonant ordering follows ``scenario_tree.build_vardatalist``
(``mpisppy/scenario_tree.py:11-42``): an indexed variable contributes its
members in ``sorted(keys)`` order, scalar variables and explicit lists keep
their order.
"""
import math

import numpy as np

minimize = 1
maximize = -1

INF = math.inf


class Var:
    """A scalar decision variable (``pyo.Var`` data analogue)."""

    __slots__ = ("model", "index", "name", "lb", "ub", "fixed", "_fixed_value")

    def __init__(self, model, index, name, lb, ub):
        self.model = model
        self.index = index
        self.name = name
        self.lb = lb
        self.ub = ub
        self.fixed = False
        self._fixed_value = None

    def is_indexed(self):
        return False

    def is_binary(self):
        return False

    # linear-expression sugar -------------------------------------------
    def __mul__(self, a):
        return LinExpr({self.index: float(a)}, 0.0, self.model)

    __rmul__ = __mul__

    def __add__(self, o):
        return LinExpr({self.index: 1.0}, 0.0, self.model) + o

    __radd__ = __add__

    def __sub__(self, o):
        return LinExpr({self.index: 1.0}, 0.0, self.model) - o

    def __rsub__(self, o):
        return (-1.0) * self + o

    def __neg__(self):
        return LinExpr({self.index: -1.0}, 0.0, self.model)

    def fix(self, value):
        self.fixed = True
        self._fixed_value = float(value)

    def unfix(self):
        self.fixed = False

    def __repr__(self):
        return "Var(%s)" % self.name


class IndexedVar:
    """An indexed variable family (``pyo.Var(Set)`` analogue)."""

    def __init__(self, model, name, keys, lb, ub):
        self.model = model
        self.name = name
        self._data = {}
        for k in keys:
            l = lb(k) if callable(lb) else (lb[k] if isinstance(lb, dict) else lb)
            u = ub(k) if callable(ub) else (ub[k] if isinstance(ub, dict) else ub)
            self._data[k] = model._new_var("%s[%s]" % (name, k), l, u)

    def is_indexed(self):
        return True

    def keys(self):
        return self._data.keys()

    def values(self):
        return self._data.values()

    def items(self):
        return self._data.items()

    def __getitem__(self, k):
        return self._data[k]

    def __iter__(self):
        return iter(self._data)

    def __len__(self):
        return len(self._data)


class LinExpr:
    """Affine expression  sum_j coef_j x_j + const."""

    __slots__ = ("coef", "const", "model")

    def __init__(self, coef=None, const=0.0, model=None):
        self.coef = dict(coef or {})
        self.const = float(const)
        self.model = model

    def _merge(self, o, sign):
        r = LinExpr(self.coef, self.const, self.model)
        if isinstance(o, LinExpr):
            for j, a in o.coef.items():
                r.coef[j] = r.coef.get(j, 0.0) + sign * a
            r.const += sign * o.const
            r.model = r.model or o.model
        elif isinstance(o, Var):
            r.coef[o.index] = r.coef.get(o.index, 0.0) + sign
            r.model = r.model or o.model
        else:
            r.const += sign * float(o)
        return r

    def __add__(self, o):
        return self._merge(o, 1.0)

    __radd__ = __add__

    def __sub__(self, o):
        return self._merge(o, -1.0)

    def __rsub__(self, o):
        return (self * -1.0) + o

    def __mul__(self, a):
        a = float(a)
        return LinExpr({j: a * v for j, v in self.coef.items()}, a * self.const, self.model)

    __rmul__ = __mul__

    def __neg__(self):
        return self * -1.0


def quicksum(terms):
    e = LinExpr()
    for t in terms:
        e = e + t
    return e


class LinearModel:
    """A scenario's LP:  min/max c'x + c0  s.t.  bl <= A x <= bu,  lb <= x <= ub.

    Single-variable rows with coefficient +-1 are folded into the variable's
    bounds, the way the reference's solvers see e.g. farmer's
    ``EnforceQuotas`` (SURVEY.md §8.0 "folded" rows).
    """

    def __init__(self, name=None):
        self.name = name
        self._vars = []
        self._rows = []          # (cols ndarray, vals ndarray, lb, ub)
        self._obj = LinExpr()
        self.sense = minimize
        self._mpisppy_node_list = None
        self._mpisppy_probability = None

    # variables ----------------------------------------------------------
    def _new_var(self, name, lb, ub):
        v = Var(self, len(self._vars), name, -INF if lb is None else float(lb),
                INF if ub is None else float(ub))
        self._vars.append(v)
        return v

    def add_var(self, name, lb=None, ub=None):
        return self._new_var(name, lb, ub)

    def add_indexed_var(self, name, keys, lb=None, ub=None):
        return IndexedVar(self, name, keys, lb, ub)

    @property
    def nvars(self):
        return len(self._vars)

    def var(self, j):
        return self._vars[j]

    # rows ---------------------------------------------------------------
    def add_constraint(self, expr, lb=None, ub=None):
        """Add ``lb <= expr <= ub`` (expr a LinExpr/Var; its constant moves right)."""
        if isinstance(expr, Var):
            expr = LinExpr({expr.index: 1.0}, 0.0, self)
        lb = -INF if lb is None else float(lb) - expr.const
        ub = INF if ub is None else float(ub) - expr.const
        items = [(j, a) for j, a in expr.coef.items() if a != 0.0]
        if len(items) == 1 and abs(items[0][1]) == 1.0:
            j, a = items[0]
            v = self._vars[j]
            lo, hi = (lb, ub) if a > 0 else (-ub, -lb)
            v.lb = max(v.lb, lo)
            v.ub = min(v.ub, hi)
            return None
        cols = np.array([j for j, _ in items], dtype=np.int64)
        vals = np.array([a for _, a in items], dtype=np.float64)
        order = np.argsort(cols, kind="stable")
        self._rows.append((cols[order], vals[order], lb, ub))
        return len(self._rows) - 1

    def add_row(self, cols, vals, lb=None, ub=None):
        """Fast path: add a row from column indices and coefficients."""
        terms = {}
        for j, a in zip(cols, vals):
            terms[int(j)] = terms.get(int(j), 0.0) + float(a)
        return self.add_constraint(LinExpr(terms, 0.0, self), lb, ub)

    # objective ----------------------------------------------------------
    def set_objective(self, expr, sense=minimize):
        if isinstance(expr, Var):
            expr = LinExpr({expr.index: 1.0}, 0.0, self)
        self._obj = expr
        self.sense = sense

    def is_minimizing(self):
        return self.sense == minimize

    # extraction ---------------------------------------------------------
    def standard_form(self):
        """Return dict(rowptr, colidx, vals, bl, bu, lb, ub, c, c0, sense)."""
        n = len(self._vars)
        m = len(self._rows)
        rowptr = np.zeros(m + 1, dtype=np.int32)
        for i, (cols, _, _, _) in enumerate(self._rows):
            rowptr[i + 1] = rowptr[i] + len(cols)
        colidx = np.concatenate([r[0] for r in self._rows]).astype(np.int32) if m else np.zeros(0, np.int32)
        vals = np.concatenate([r[1] for r in self._rows]) if m else np.zeros(0)
        bl = np.array([r[2] for r in self._rows], dtype=np.float64)
        bu = np.array([r[3] for r in self._rows], dtype=np.float64)
        lb = np.array([v.lb for v in self._vars], dtype=np.float64)
        ub = np.array([v.ub for v in self._vars], dtype=np.float64)
        for v in self._vars:
            if v.fixed:
                lb[v.index] = ub[v.index] = v._fixed_value
        c = np.zeros(n)
        for j, a in self._obj.coef.items():
            c[j] += a
        return dict(rowptr=rowptr, colidx=colidx, vals=vals, bl=bl, bu=bu, lb=lb, ub=ub,
                    c=c, c0=self._obj.const, sense=self.sense)


def build_vardatalist(varlist):
    """Expand a nonant list the way ``scenario_tree.build_vardatalist`` does
    (``mpisppy/scenario_tree.py:28-42``): indexed members in sorted(keys)."""
    if isinstance(varlist, (Var, IndexedVar)):
        varlist = [varlist]
    out = []
    for v in varlist:
        if isinstance(v, IndexedVar):
            out.extend(v[k] for k in sorted(v.keys()))
        elif isinstance(v, (list, tuple)):
            out.extend(v)
        else:
            out.append(v)
    return out
