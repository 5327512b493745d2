"""A small linear modelling layer standing in for a Pyomo ConcreteModel.

The reference's scenario creators return Pyomo models; the hot path only
ever needs their standard linear representation (``pyomo.repn``), which
the batched layout extracts once.  Pyomo is not part of this image, so the
examples build a :class:`LinearModel` instead, and :mod:`mpisppy_amd.repn`
converts a real Pyomo model when Pyomo is importable.

Semantics kept from Pyomo that matter for PH parity:
* indexed variables remember their index keys; ``sorted(keys)`` gives the
  nonant order (``mpisppy/scenario_tree.py:36``);
* a constraint ``lo <= expr <= hi`` with constants moved to the bounds;
* the objective sense (maximize models are negated into min form by the
  layout, ``phbase.py:1206-1209``).
"""
import math
import numpy as np
import scipy.sparse as sp

INF = math.inf


class LinExpr:
    """Linear expression: {column: coefficient} + constant."""
    __slots__ = ("terms", "const")

    def __init__(self, terms=None, const=0.0):
        self.terms = dict(terms) if terms else {}
        self.const = float(const)

    @staticmethod
    def of(v):
        if isinstance(v, LinExpr):
            return v
        if isinstance(v, VarData):
            return LinExpr({v.col: 1.0})
        if isinstance(v, Var):
            return LinExpr({v._scalar().col: 1.0})
        return LinExpr(None, float(v))

    def copy(self):
        return LinExpr(self.terms, self.const)

    def __add__(self, o):
        o = LinExpr.of(o)
        r = self.copy()
        for k, v in o.terms.items():
            r.terms[k] = r.terms.get(k, 0.0) + v
        r.const += o.const
        return r

    __radd__ = __add__

    def __neg__(self):
        return LinExpr({k: -v for k, v in self.terms.items()}, -self.const)

    def __sub__(self, o):
        return self + (-LinExpr.of(o))

    def __rsub__(self, o):
        return LinExpr.of(o) - self

    def __mul__(self, a):
        a = float(a)
        return LinExpr({k: a * v for k, v in self.terms.items()}, a * self.const)

    __rmul__ = __mul__

    def __le__(self, o):
        return _Rel(self - LinExpr.of(o), -INF, 0.0)

    def __ge__(self, o):
        return _Rel(self - LinExpr.of(o), 0.0, INF)

    def __eq__(self, o):  # noqa: D105 -- builds an equality relation
        return _Rel(self - LinExpr.of(o), 0.0, 0.0)

    __hash__ = None


class _Rel:
    def __init__(self, expr, lo, hi):
        self.expr, self.lo, self.hi = expr, lo, hi


class VarData:
    """One scalar variable (a Pyomo _GeneralVarData analogue)."""
    __slots__ = ("model", "col", "name")

    def __init__(self, model, col, name):
        self.model, self.col, self.name = model, col, name

    def _e(self):
        return LinExpr({self.col: 1.0})

    def __add__(self, o): return self._e() + o
    def __radd__(self, o): return self._e() + o
    def __sub__(self, o): return self._e() - o
    def __rsub__(self, o): return LinExpr.of(o) - self._e()
    def __mul__(self, a): return self._e() * a
    __rmul__ = __mul__
    def __neg__(self): return -self._e()
    def __le__(self, o): return self._e() <= o
    def __ge__(self, o): return self._e() >= o
    def __eq__(self, o): return self._e() == o
    __hash__ = object.__hash__

    def is_indexed(self):
        return False

    @property
    def lb(self):
        return self.model._lb[self.col]

    @property
    def ub(self):
        return self.model._ub[self.col]

    @property
    def value(self):
        v = self.model._values
        return None if v is None else float(v[self.col])


class Var:
    """Indexed (or scalar when index is None) variable block."""

    def __init__(self, model, name, index, lb, ub):
        self.model, self.name = model, name
        self._data = {}
        keys = [None] if index is None else list(index)
        for key in keys:
            nm = name if key is None else f"{name}[{key}]"
            lo = lb(key) if callable(lb) else lb
            hi = ub(key) if callable(ub) else ub
            col = model._new_col(nm, -INF if lo is None else lo, INF if hi is None else hi)
            self._data[key] = VarData(model, col, nm)
        self._indexed = index is not None

    def is_indexed(self):
        return self._indexed

    def keys(self):
        return list(self._data.keys())

    def __getitem__(self, key):
        return self._data[key]

    def __iter__(self):
        return iter(self._data.keys())

    def values(self):
        return list(self._data.values())

    # scalar var convenience
    def _scalar(self):
        if self._indexed:
            raise TypeError(f"{self.name} is indexed")
        return self._data[None]

    def __add__(self, o): return self._scalar() + o
    def __radd__(self, o): return self._scalar() + o
    def __sub__(self, o): return self._scalar() - o
    def __rsub__(self, o): return o - self._scalar()
    def __mul__(self, a): return self._scalar() * a
    __rmul__ = __mul__
    def __neg__(self): return -self._scalar()
    def __le__(self, o): return self._scalar() <= o
    def __ge__(self, o): return self._scalar() >= o
    def __eq__(self, o): return self._scalar() == o
    __hash__ = object.__hash__


class LinearModel:
    """Scenario LP container: variables, ranged rows and one objective."""

    def __init__(self, name="model"):
        self.name = name
        self._names, self._lb, self._ub = [], [], []
        self._rows = []      # (name, terms dict, lo, hi)
        self._obj = LinExpr()
        self.sense = "min"
        self._values = None
        self._exprs = {}

    # -- building ----------------------------------------------------------
    def _new_col(self, name, lb, ub):
        self._names.append(name)
        self._lb.append(float(lb))
        self._ub.append(float(ub))
        return len(self._names) - 1

    def add_var(self, name, index=None, lb=None, ub=None):
        v = Var(self, name, index, lb, ub)
        setattr(self, name, v)
        return v if index is not None else v

    def add_constraint(self, name, rel, lo=None, hi=None):
        """Add ``rel`` (``a <= b``, ``a >= b``, ``a == b``) or, with lo/hi,
        the ranged row ``lo <= rel <= hi`` where ``rel`` is an expression."""
        if isinstance(rel, _Rel):
            e, lo_, hi_ = rel.expr, rel.lo, rel.hi
        else:
            e = LinExpr.of(rel)
            lo_ = -INF if lo is None else float(lo)
            hi_ = INF if hi is None else float(hi)
        terms = {k: v for k, v in e.terms.items()}
        self._rows.append((name, terms, lo_ - e.const, hi_ - e.const))

    def set_objective(self, expr, sense="min"):
        if sense not in ("min", "max"):
            raise ValueError("Model sense Not recognized")
        self._obj = LinExpr.of(expr)
        self.sense = sense

    def add_expression(self, name, expr):
        self._exprs[name] = LinExpr.of(expr)
        setattr(self, name, self._exprs[name])
        return self._exprs[name]

    # -- extraction (the "standard repn") -----------------------------------
    @property
    def num_vars(self):
        return len(self._names)

    def standard_form(self):
        """Return dict(c, const, A(csr), rl, ru, l, u, var_names, row_names, sense)
        of  opt c'x + const  s.t. rl <= A x <= ru, l <= x <= u  (model sense)."""
        n = len(self._names)
        c = np.zeros(n)
        for k, v in self._obj.terms.items():
            c[k] += v
        indptr = [0]
        indices, data, rl, ru, rnames = [], [], [], [], []
        for name, terms, lo, hi in self._rows:
            cols = sorted(terms)
            indices.extend(cols)
            data.extend(terms[j] for j in cols)
            indptr.append(len(indices))
            rl.append(lo)
            ru.append(hi)
            rnames.append(name)
        A = sp.csr_matrix((np.asarray(data, dtype=np.float64),
                           np.asarray(indices, dtype=np.int64),
                           np.asarray(indptr, dtype=np.int64)), shape=(len(self._rows), n))
        return dict(c=c, const=self._obj.const, A=A, rl=np.asarray(rl, dtype=np.float64),
                    ru=np.asarray(ru, dtype=np.float64), l=np.asarray(self._lb),
                    u=np.asarray(self._ub), var_names=list(self._names), row_names=rnames,
                    sense=self.sense)

    def load_values(self, x):
        """Attach solution values (read back by VarData.value)."""
        self._values = np.asarray(x, dtype=np.float64)


def value(e, model=None):
    """pyo.value analogue for LinExpr / VarData on a model with loaded values."""
    if isinstance(e, VarData):
        return e.value
    if isinstance(e, LinExpr):
        if model is None:
            raise ValueError("model required to evaluate an expression")
        x = model._values
        return e.const + sum(v * x[k] for k, v in e.terms.items())
    return float(e)
