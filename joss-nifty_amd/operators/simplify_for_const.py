"""Constant-input insertion (src/operators/simplify_for_const.py:110-138).

``InsertionOperator(target, cst)`` maps the variable keys of ``target`` to the
full MultiDomain by uniting with the constant MultiField ``cst``; its Jacobian
is the embedding var -> full (zero on the constant keys), i.e. the adjoint of
the PartialExtractor full -> var."""
from ..multi_domain import MultiDomain
from ..multi_field import MultiField
from .operator import Operator


class InsertionOperator(Operator):
    def __init__(self, target, cst_field):
        from .simple_linear_operators import PartialExtractor
        if not isinstance(target, MultiDomain):
            raise TypeError
        if not isinstance(cst_field, MultiField):
            raise TypeError
        self._target = MultiDomain.make(target)
        self._cst = cst_field
        dom = {kk: vv for kk, vv in self._target.items() if kk not in cst_field.keys()}
        self._domain = MultiDomain.make(dom)
        self._jac = PartialExtractor(self._target, self._domain).adjoint

    def apply(self, x):
        self._check_input(x)
        val = x if x.jac is None else x.val
        if set(self._cst.keys()) & set(val.domain.keys()):
            raise ValueError("constant and variable keys overlap")
        val = val.unite(self._cst)
        if val.domain is not self._target:
            val = MultiField(self._target, tuple(val[k] for k in self._target.keys()))
        if x.jac is None:
            return val
        return x.new(val, self._jac)

    def __repr__(self):
        return f"InsertionOperator\n  Constant: {self._cst.keys()}\n  Variable: {self._domain.keys()}"
