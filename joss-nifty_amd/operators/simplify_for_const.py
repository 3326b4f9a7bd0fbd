"""Minimal constant-input insertion (src/operators/simplify_for_const.py)."""
from ..multi_domain import MultiDomain
from .operator import Operator


class InsertionOperator(Operator):
    def __init__(self, target, cst_field):
        self._target = target
        self._cst = cst_field
        dom = {kk: vv for kk, vv in target.items() if kk not in cst_field.keys()}
        self._domain = MultiDomain.make(dom)

    def apply(self, x):
        self._check_input(x)
        if x.jac is not None:
            raise NotImplementedError("constant insertion under Linearization is a 'next' item")
        return x.unite(self._cst)
