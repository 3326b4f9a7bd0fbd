"""Adder: x -> x + a (or x - a) (src/operators/adder.py)."""
import numpy as np

from ..field import Field
from ..multi_field import MultiField
from .operator import Operator


class Adder(Operator):
    def __init__(self, a, neg=False, domain=None):
        from ..sugar import makeDomain, makeField
        self._a = a
        if isinstance(a, (Field, MultiField)):
            dom = a.domain
        elif np.isscalar(a):
            dom = makeDomain(domain)
        else:
            raise TypeError
        self._domain = self._target = dom
        self._neg = bool(neg)

    def apply(self, x):
        self._check_input(x)
        if x.jac is not None:
            return x.new(x.val - self._a if self._neg else x.val + self._a, x.jac)
        return x - self._a if self._neg else x + self._a
