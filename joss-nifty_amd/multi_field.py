"""MultiField: Fields keyed by the sorted keys of a MultiDomain
(src/multi_field.py:26-396)."""
import numpy as np
import torch

from . import utilities
from .field import Field
from .multi_domain import MultiDomain


class MultiField:
    def __init__(self, domain, val):
        if not isinstance(domain, MultiDomain):
            raise TypeError("domain must be of type MultiDomain")
        if not isinstance(val, tuple):
            raise TypeError("values must be a tuple")
        if len(val) != len(domain):
            raise ValueError("length mismatch")
        for d, v in zip(domain._domains, val):
            if isinstance(v, Field):
                if v._domain != d:
                    raise ValueError("domain mismatch")
            else:
                raise TypeError("bad entry in tuple of fields")
        self._domain = domain
        self._val = val

    @staticmethod
    def from_dict(dct, domain=None):
        if domain is None:
            for k, v in dct.items():
                if not isinstance(v, Field):
                    raise TypeError("Value must be a Field")
            domain = MultiDomain.make({key: v._domain for key, v in dct.items()})
        res = tuple(dct[key] if key in dct else Field(dom, torch.zeros(dom.shape, dtype=torch.float64,
                                                                        device=_dev()))
                    for key, dom in zip(domain.keys(), domain.domains()))
        return MultiField(domain, res)

    def to_dict(self):
        return {key: val for key, val in zip(self._domain.keys(), self._val)}

    def __getitem__(self, key):
        return self._val[self._domain.idx[key]]

    def __contains__(self, key):
        return key in self._domain.idx

    def keys(self):
        return self._domain.keys()

    def items(self):
        return zip(self._domain.keys(), self._val)

    def values(self):
        return self._val

    @property
    def domain(self):
        return self._domain

    @property
    def dtype(self):
        return {key: val.dtype for key, val in self.items()}

    def _transform(self, op):
        return MultiField(self._domain, tuple(op(v) for v in self._val))

    @property
    def real(self):
        return self._transform(lambda x: x.real)

    @property
    def imag(self):
        return self._transform(lambda x: x.imag)

    @staticmethod
    def from_random(domain, random_type="normal", dtype=np.float64, **kwargs):
        """Keys drawn in sorted order (multi_field.py:103-127)."""
        domain = MultiDomain.make(domain)
        if isinstance(dtype, dict):
            dtype = {kk: dtype[kk] for kk in domain.keys()}
        else:
            dtype = {kk: dtype for kk in domain.keys()}
        dct = {kk: Field.from_random(domain[kk], random_type, dtype[kk], **kwargs) for kk in domain.keys()}
        return MultiField.from_dict(dct, domain)

    def s_vdot(self, x):
        """Sum of the per-key Field.s_vdot values in key order.  The per-key
        device reductions are the same; their results come to the host in ONE
        copy instead of one synchronising .item() per key."""
        if len(self._val) < 2:
            return sum(v1.s_vdot(v2) for v1, v2 in zip(self._val, x._val))
        from .ducc_dispatch import vdot
        parts = []
        for v1, v2 in zip(self._val, x._val):
            if not isinstance(v2, Field):
                raise TypeError("The dot-partner must be an instance of the Field class")
            utilities.check_object_identity(v2._domain, v1._domain)
            parts.append(vdot(v1._val, v2._val))
        if any(t.is_complex() for t in parts):
            return sum(t.item() for t in parts)
        return sum(torch.stack(parts).tolist())

    def vdot(self, x):
        return Field.scalar(self.s_vdot(x))

    def dev_vdot(self, x):
        """Sum of per-key dots as a 0-d device tensor (no host sync)."""
        from .ducc_dispatch import vdot
        res = None
        for v1, v2 in zip(self._val, x._val):
            t = vdot(v1.val, v2.val)
            res = t if res is None else res + t
        return res

    @staticmethod
    def full(domain, val):
        domain = MultiDomain.make(domain)
        return MultiField(domain, tuple(Field.full(dom, val) for dom in domain._domains))

    @property
    def val(self):
        return {key: val.val for key, val in zip(self._domain.keys(), self._val)}

    def val_rw(self):
        return {key: val.val_rw() for key, val in zip(self._domain.keys(), self._val)}

    @staticmethod
    def from_raw(domain, arr):
        return MultiField(domain, tuple(Field(domain[key], arr[key]) for key in domain.keys()))

    def norm(self, ord=2):
        if ord == 2:
            s = self.dev_vdot(self).real.item()
            return float(np.sqrt(max(s, 0.)))
        return float(np.linalg.norm(np.array([f.norm(ord=ord) for f in self._val]), ord=ord))

    def s_sum(self):
        return sum(v.s_sum() for v in self._val)

    @property
    def size(self):
        return sum(v.size for v in self._val)

    def __neg__(self):
        return self._transform(lambda x: -x)

    def __abs__(self):
        return self._transform(lambda x: abs(x))

    def conjugate(self):
        return self._transform(lambda x: x.conjugate())

    def clip(self, a_min=None, a_max=None):
        return self._transform(lambda x: x.clip(a_min, a_max))

    def s_all(self):
        return all(v.s_all() for v in self._val)

    def s_any(self):
        return any(v.s_any() for v in self._val)

    def extract(self, subset):
        if subset is self._domain:
            return self
        return MultiField(subset, tuple(self[key] for key in subset.keys()))

    def extract_by_keys(self, keys):
        dom = MultiDomain.make({kk: vv for kk, vv in self.domain.items() if kk in keys})
        return self.extract(dom)

    def extract_part(self, subset):
        if subset is self._domain:
            return self
        return MultiField.from_dict({key: self[key] for key in subset.keys() if key in self})

    def unite(self, other):
        if self._domain is other._domain:
            return self + other
        res = self.to_dict()
        for key, val in other.items():
            res[key] = res[key] + val if key in res else val
        return MultiField.from_dict(res)

    @staticmethod
    def union(fields, domain=None):
        res = {}
        for field in fields:
            res.update(field.to_dict())
        return MultiField.from_dict(res, domain)

    def flexible_addsub(self, other, neg):
        if self._domain is other._domain:
            return self - other if neg else self + other
        res = self.to_dict()
        for key, val in other.items():
            if key in res:
                res[key] = res[key] - val if neg else res[key] + val
            else:
                res[key] = -val if neg else val
        return MultiField.from_dict(res)

    def ptw(self, op, *args, **kwargs):
        return self._transform(lambda x: x.ptw(op, *args, **kwargs))

    def ptw_with_deriv(self, op, *args, **kwargs):
        tmp = [v.ptw_with_deriv(op, *args, **kwargs) for v in self._val]
        return (MultiField(self._domain, tuple(v[0] for v in tmp)),
                MultiField(self._domain, tuple(v[1] for v in tmp)))

    def _binary_op(self, other, op):
        if isinstance(other, MultiField):
            if self._domain != other._domain:
                raise ValueError("domain mismatch")
            return MultiField(self._domain, tuple(getattr(v1, op)(v2) for v1, v2 in zip(self._val, other._val)))
        if np.isscalar(other) or (isinstance(other, torch.Tensor) and other.ndim == 0):
            return self._transform(lambda x: getattr(x, op)(other))
        return NotImplemented

    def __repr__(self):
        return "<nifty_amd.MultiField>"


def _dev():
    from . import config
    return config.device()


for _op in ["__add__", "__radd__", "__sub__", "__rsub__", "__mul__", "__rmul__", "__truediv__",
            "__rtruediv__", "__floordiv__", "__rfloordiv__", "__pow__", "__rpow__", "__lt__", "__le__",
            "__gt__", "__ge__", "__eq__", "__ne__"]:
    setattr(MultiField, _op, (lambda op: lambda self, other: self._binary_op(other, op))(_op))
MultiField.__hash__ = None
for _f in ("sqrt", "exp", "log", "tanh", "sigmoid", "reciprocal", "absolute"):
    setattr(MultiField, _f, (lambda name: lambda self: self.ptw(name))(_f))

MultiField.jac = None
MultiField.want_metric = False
MultiField.metric = None
