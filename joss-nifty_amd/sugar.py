"""Convenience constructors (subset of src/sugar.py on the sampling path)."""
import numpy as np
import torch

from . import utilities
from .domain_tuple import DomainTuple
from .field import Field
from .multi_domain import MultiDomain
from .multi_field import MultiField


def makeDomain(domain):
    if isinstance(domain, (MultiDomain, dict)):
        return MultiDomain.make(domain)
    return DomainTuple.make(domain)


def makeField(domain, arr):
    if isinstance(domain, (dict, MultiDomain)):
        return MultiField.from_raw(makeDomain(domain), arr)
    return Field.from_raw(makeDomain(domain), arr)


def full(domain, val):
    if isinstance(domain, (dict, MultiDomain)):
        return MultiField.full(domain, val)
    return Field.full(domain, val)


def from_random(domain, random_type="normal", dtype=np.float64, **kwargs):
    domain = makeDomain(domain)
    if isinstance(domain, MultiDomain):
        return MultiField.from_random(domain, random_type, dtype, **kwargs)
    return Field.from_random(domain, random_type, dtype, **kwargs)


def makeOp(inp, dom=None, sampling_dtype=None):
    from .operators.block_diagonal_operator import BlockDiagonalOperator
    from .operators.diagonal_operator import DiagonalOperator
    from .operators.scaling_operator import ScalingOperator
    if inp is None:
        return None
    if np.isscalar(inp):
        if not isinstance(dom, (DomainTuple, MultiDomain)):
            raise TypeError("need proper `dom` argument")
        return ScalingOperator(dom, inp, sampling_dtype=sampling_dtype)
    if dom is not None:
        utilities.check_object_identity(dom, inp.domain)
    if inp.domain is DomainTuple.scalar_domain():
        return ScalingOperator(inp.domain, inp.val.item(), sampling_dtype=sampling_dtype)
    if isinstance(inp, Field):
        return DiagonalOperator(inp, sampling_dtype=sampling_dtype)
    if isinstance(inp, MultiField):
        dct = {}
        for key, val in inp.items():
            sdt = sampling_dtype[key] if isinstance(sampling_dtype, dict) else sampling_dtype
            dct[key] = makeOp(val, sampling_dtype=sdt)
        return BlockDiagonalOperator(inp.domain, dct)
    raise NotImplementedError


def domain_union(domains):
    if isinstance(domains[0], DomainTuple):
        for dom in domains[1:]:
            utilities.check_object_identity(dom, domains[0])
        return domains[0]
    return MultiDomain.union(domains)


def is_operator(obj):
    from .operators.operator import Operator
    return isinstance(obj, Operator) and not is_fieldlike(obj)


def is_linearization(obj):
    from .linearization import Linearization
    return isinstance(obj, Linearization)


def is_fieldlike(obj):
    return isinstance(obj, (Field, MultiField))


def _ptw_op(name):
    def f(x):
        return x.ptw(name)
    f.__name__ = name
    return f


for _name in ["sqrt", "exp", "log", "sin", "cos", "tan", "sinh", "cosh", "tanh", "sinc", "sigmoid",
              "absolute", "reciprocal", "log10", "log1p", "expm1", "softplus", "arctan"]:
    globals()[_name] = _ptw_op(_name)
