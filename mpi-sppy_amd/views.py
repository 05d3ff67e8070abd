"""Host views of the device-resident PH state, per local scenario.

Extensions, convergers, rho setters and denouement callbacks of the reference
read and write PH state through each scenario's Pyomo objects:
``s._mpisppy_model.{W, xbars, xsqbars, rho, W_on, prox_on}``, nonant Var values
via ``s._mpisppy_data.nonant_indices`` and ``s._mpisppy_data.{nlens, prob_coeff,
outer_bound, inner_bound, scenario_feasible}``.  Here those
attributes are light views onto the batched device tensors: reads copy the
device array to the host once per device update (``SPBase._host``), writes to
W / rho go straight to the device.  Nothing is materialised unless a hook asks.
"""
from collections.abc import Mapping



class _ParamData:
    __slots__ = ("_get", "_set")

    def __init__(self, get, set_=None):
        self._get = get
        self._set = set_

    @property
    def value(self):
        return self._get()

    @value.setter
    def value(self, v):
        if self._set is None:
            raise AttributeError("read-only PH quantity")
        self._set(v)

    _value = value

    def __float__(self):
        return float(self._get())


class _Param:
    """Indexed by the reference's nonant key (ndn, i)."""

    def __init__(self, view, key):
        self._view = view
        self._key = key

    def _slot(self, ndn_i):
        return self._view._slot_of_key(ndn_i)

    def __getitem__(self, ndn_i):
        v = self._view
        j = self._slot(ndn_i)
        opt = v._opt
        if self._key in ("W", "rho"):
            return _ParamData(lambda: float(opt._host(self._key)[j, v._s]),
                              lambda val: opt._host_write(self._key, j, v._s, val))
        arr_key = "xbar" if self._key == "xbars" else "xsqbar"
        idx = int(opt._xbar_idx[j, v._s])
        return _ParamData(lambda: float(opt._host(arr_key)[idx]))

    def __setitem__(self, ndn_i, val):
        if self._key not in ("W", "rho"):
            raise AttributeError("xbars are computed by Compute_Xbar")
        j = self._slot(ndn_i)
        self._view._opt._host_write(self._key, j, self._view._s, val)

    def keys(self):
        return self._view._keys()

    def __iter__(self):
        return iter(self._view._keys())

    def __len__(self):
        return len(self._view._keys())


class _Flag:
    def __init__(self, opt, attr):
        self._opt = opt
        self._attr = attr

    @property
    def value(self):
        return getattr(self._opt, self._attr)

    @value.setter
    def value(self, v):
        setattr(self._opt, self._attr, int(v))

    _value = value


class _VarView:
    """A nonant variable of one scenario (Pyomo VarData stand-in)."""

    __slots__ = ("_opt", "_s", "_col", "name")

    def __init__(self, opt, s, col, name):
        self._opt = opt
        self._s = s
        self._col = col
        self.name = name

    def _slot(self):
        return int(list(self._opt.batch.nonant.slot_col).index(self._col))

    @property
    def value(self):
        return float(self._opt._host("x")[self._col, self._s])

    @value.setter
    def value(self, v):
        self._opt._host_write("x", self._col, self._s, v)

    _value = value

    def set_value(self, v):
        self.value = v

    @property
    def fixed(self):
        f = getattr(self._opt, "_fixed", None)
        return bool(f is not None and f[self._s, self._slot()])

    @fixed.setter
    def fixed(self, flag):
        if flag:
            self.fix()
        else:
            self.unfix()

    def is_fixed(self):
        return self.fixed

    def fix(self, value=None):
        """Fix at ``value`` (or the current value), like Pyomo's VarData.fix."""
        opt = self._opt
        fixed, fv = opt._fix_arrays()
        j = self._slot()
        v = self.value if value is None else float(value)
        if value is not None:
            self.value = v
        fixed[self._s, j] = True
        fv[self._s, j] = v
        opt._fix_dirty = True

    def unfix(self):
        opt = self._opt
        fixed, _ = opt._fix_arrays()
        j = self._slot()
        if fixed[self._s, j]:
            fixed[self._s, j] = False
            opt._fix_dirty = True

    @property
    def stale(self):
        return False

    def is_binary(self):
        return False

    def is_integer(self):
        return False


class _ModelNS:
    def __init__(self, view):
        opt = view._opt
        self.W = _Param(view, "W")
        self.rho = _Param(view, "rho")
        self.xbars = _Param(view, "xbars")
        self.xsqbars = _Param(view, "xsqbars")
        self.W_on = _Flag(opt, "W_on")
        self.prox_on = _Flag(opt, "prox_on")


class _DataNS:
    def __init__(self, view):
        self._view = view

    @property
    def nonant_indices(self):
        v = self._view
        opt = v._opt
        nn = opt.batch.nonant
        return {k: _VarView(opt, v._s, int(nn.slot_col[j]), nn.var_names[j])
                for j, k in enumerate(v._keys())}

    @property
    def nlens(self):
        v = self._view
        out = {}
        for (ndn, i) in v._keys():
            out[ndn] = out.get(ndn, 0) + 1
        return out

    @property
    def prob_coeff(self):
        v = self._view
        opt = v._opt
        out = {}
        for j, (ndn, i) in enumerate(v._keys()):
            out.setdefault(ndn, float(opt._prob_coeff[j, v._s]))
        return out

    @property
    def outer_bound(self):
        return float(self._view._opt._host("outer")[self._view._s])

    @property
    def inner_bound(self):
        return self.outer_bound

    @property
    def scenario_feasible(self):
        return int(self._view._opt._host("status")[self._view._s]) == 1

    @property
    def has_variable_probability(self):
        return False

    # per-scenario rows of the opt's [S_local][N] caches (writable numpy views)
    def _cache_row(self, name):
        a = getattr(self._view._opt, name, None)
        return None if a is None else a[self._view._s]

    @property
    def nonant_cache(self):
        return self._cache_row("nonant_cache")

    @property
    def fixedness_cache(self):
        return self._cache_row("fixedness_cache")

    @property
    def original_nonants(self):
        return self._cache_row("original_nonants")

    @property
    def original_fixedness(self):
        return self._cache_row("original_fixedness")


class ScenarioView:
    """One local scenario as seen by hooks (``local_scenarios[name]``)."""

    def __init__(self, opt, s, name):
        self._opt = opt
        self._s = s
        self.name = name
        self._keys_cache = None
        self._mpisppy_model = _ModelNS(self)
        self._mpisppy_data = _DataNS(self)

    @property
    def _mpisppy_probability(self):
        return float(self._opt.batch.prob[self._s])

    def _keys(self):
        if self._keys_cache is None:
            self._keys_cache = self._opt.slot_keys(self._s)
        return self._keys_cache

    def _slot_of_key(self, ndn_i):
        try:
            return self._keys().index(tuple(ndn_i))
        except ValueError:
            raise KeyError(ndn_i)

    def _slot_of_varid(self, vid):
        models = self._opt._models
        if models is None:
            raise RuntimeError("rho_setter needs per-scenario models (options['per_scenario_models']=True)")
        mdl = models[self.name]
        cols = list(self._opt.batch.nonant.slot_col)
        for v in mdl._vars:
            if id(v) == vid:
                return cols.index(v.index)
        raise KeyError(vid)

    @property
    def model(self):
        m = self._opt._models
        return None if m is None else m[self.name]


class ScenarioViews(Mapping):
    """``local_scenarios``: name -> ScenarioView, each built on first access.
    A million local scenarios cost ~20 us of Python objects each when built
    eagerly (20 s at 1M); the engine itself never needs them, only hooks and
    callers that index or iterate the dict do."""

    def __init__(self, opt, names):
        self._opt = opt
        self._names = list(names)
        self._index = None
        self._built = {}

    def _k(self, name):
        if self._index is None:
            self._index = {nm: k for k, nm in enumerate(self._names)}
        return self._index[name]

    def __getitem__(self, name):
        v = self._built.get(name)
        if v is None:
            v = self._built[name] = ScenarioView(self._opt, self._k(name), name)
        return v

    def __iter__(self):
        return iter(self._names)

    def __len__(self):
        return len(self._names)

    def __contains__(self, name):
        try:
            self._k(name)
            return True
        except (KeyError, TypeError):
            return False
