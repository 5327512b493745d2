"""Standard-form extraction of a scenario model ("the standard repn").

* :class:`mpisppy_amd.model.LinearModel` -> its own ``standard_form()``.
* A Pyomo ConcreteModel (when Pyomo is importable; it is not in this image)
  -> ``pyomo.repn.standard_repn.generate_standard_repn`` over the active
  objective and constraints, the same representation Pyomo's LP writers and
  persistent solver plugins use (``phbase.py:903-915`` re-walks it every
  solve; here it is walked once).  This adapter is untested in this
  container because Pyomo is absent.
"""
import numpy as np
import scipy.sparse as sp

from .model import LinearModel, VarData


def _is_pyomo(model):
    return type(model).__module__.startswith("pyomo")


def standard_form(model):
    if isinstance(model, LinearModel):
        return model.standard_form()
    if _is_pyomo(model):
        return _pyomo_standard_form(model)
    raise TypeError(f"cannot extract a linear model from {type(model)!r}")


def column_of(model, vardata):
    if isinstance(model, LinearModel):
        if isinstance(vardata, VarData):
            return vardata.col
        raise TypeError("nonant is not a VarData of this model")
    cols = model.__dict__.setdefault("_mpisppy_amd_cols", None)
    if cols is None:
        raise RuntimeError("standard_form must run before column_of on a Pyomo model")
    return cols[id(vardata)]


def _pyomo_standard_form(model):  # pragma: no cover - Pyomo absent in this image
    import pyomo.environ as pyo
    from pyomo.repn.standard_repn import generate_standard_repn

    cols = {}
    names, lb, ub = [], [], []

    def col(v):
        k = id(v)
        if k not in cols:
            cols[k] = len(names)
            names.append(v.name)
            lo, hi = v.bounds
            if v.is_fixed():
                lo = hi = v.value
            lb.append(-np.inf if lo is None else float(lo))
            ub.append(np.inf if hi is None else float(hi))
        return cols[k]

    objs = list(model.component_data_objects(pyo.Objective, active=True, descend_into=True))
    if len(objs) != 1:
        raise RuntimeError("expected exactly one active objective")
    obj = objs[0]
    orep = generate_standard_repn(obj.expr, quadratic=False)
    rows, rcols, rvals, rl, ru, rnames = [], [], [], [], [], []
    for r, con in enumerate(model.component_data_objects(pyo.Constraint, active=True,
                                                         descend_into=True, sort=True)):
        rep = generate_standard_repn(con.body, quadratic=False)
        if not rep.is_linear():
            raise RuntimeError(f"constraint {con.name} is not linear")
        for v, a in zip(rep.linear_vars, rep.linear_coefs):
            rows.append(len(rl)); rcols.append(col(v)); rvals.append(float(a))
        lo = -np.inf if con.lower is None else pyo.value(con.lower) - rep.constant
        hi = np.inf if con.upper is None else pyo.value(con.upper) - rep.constant
        rl.append(lo); ru.append(hi); rnames.append(con.name)
    c_terms = [(col(v), float(a)) for v, a in zip(orep.linear_vars, orep.linear_coefs)]
    n = len(names)
    c = np.zeros(n)
    for j, a in c_terms:
        c[j] += a
    A = sp.csr_matrix((rvals, (rows, rcols)), shape=(len(rl), n))
    A.sum_duplicates()
    A.sort_indices()
    model.__dict__["_mpisppy_amd_cols"] = cols
    return dict(c=c, const=float(orep.constant), A=A, rl=np.asarray(rl), ru=np.asarray(ru),
                l=np.asarray(lb), u=np.asarray(ub), var_names=names, row_names=rnames,
                sense="min" if obj.is_minimizing() else "max")
