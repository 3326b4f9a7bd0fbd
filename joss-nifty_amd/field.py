"""Field: immutable device tensor + DomainTuple (src/field.py:28-741).

Values live in HBM as torch tensors (``.val``).  ``np.asarray(field)`` /
``field.val_np()`` give a host copy.  Reductions on the hot path (vdot, norm)
go through the native deterministic fp64 reduction (ducc_dispatch.vdot)."""
import numpy as np
import torch

from . import config, utilities
from .domain_tuple import DomainTuple


def _to_tensor(val, dtype=None):
    if isinstance(val, torch.Tensor):
        return val if dtype is None else val.to(utilities.torch_dtype(dtype))
    if isinstance(val, Field):
        return val.val
    arr = np.asarray(val)
    if dtype is not None:
        arr = arr.astype(utilities.numpy_dtype(utilities.torch_dtype(dtype)), copy=False)
    if arr.dtype == np.float16:
        arr = arr.astype(np.float32)
    dev = torch.device(config.device())
    if dev.type == "cuda":
        # a prefetched draw in page-locked memory (random._pin): async DMA
        from .random import take_pinned
        t = take_pinned(arr)
        if t is not None:
            return t.to(dev, non_blocking=True)
        if arr.ndim > 0 and arr.flags.c_contiguous and arr.flags.writeable:
            return torch.from_numpy(arr).to(dev)    # the upload is the copy
    # (np.ascontiguousarray would promote 0-d arrays to 1-d)
    return torch.from_numpy(np.array(arr, order="C", copy=True)).to(dev)


class Field:
    def __init__(self, domain, val):
        if not isinstance(domain, DomainTuple):
            raise TypeError("domain must be of type DomainTuple")
        if not isinstance(val, torch.Tensor):
            a = np.asarray(val)
            if a.shape == () and domain.shape != ():
                a = np.broadcast_to(a, domain.shape)
            val = _to_tensor(a)
        if domain.shape != tuple(val.shape):
            raise ValueError(f"shape mismatch between val and domain: {tuple(val.shape)} {domain.shape}")
        self._domain = domain
        self._val = val

    # ------------------------------------------------------------ factories
    @staticmethod
    def scalar(val):
        return Field(DomainTuple.scalar_domain(), val if isinstance(val, torch.Tensor)
                     else torch.tensor(val, device=config.device(),
                                       dtype=torch.complex128 if np.iscomplexobj(val) else torch.float64))

    @staticmethod
    def full(domain, val):
        if not np.isscalar(val) and not (isinstance(val, torch.Tensor) and val.ndim == 0):
            raise TypeError("val must be a scalar")
        domain = DomainTuple.make(domain)
        if isinstance(val, torch.Tensor):
            return Field(domain, val.expand(domain.shape).clone())
        dt = utilities.torch_dtype(np.asarray(val).dtype)  # numpy's np.full dtype rule
        return Field(domain, torch.full(domain.shape, val, dtype=dt, device=config.device()))

    @staticmethod
    def from_raw(domain, arr):
        return Field(DomainTuple.make(domain), arr)

    def cast_domain(self, new_domain):
        return Field(DomainTuple.make(new_domain), self._val)

    @staticmethod
    def from_random(domain, random_type="normal", dtype=np.float64, **kwargs):
        """Host numpy draw (bit-identical to the reference stream, field.py:133-156),
        uploaded to the device."""
        from .random import Random
        domain = DomainTuple.make(domain)
        gen = getattr(Random, random_type)
        arr = gen(dtype=dtype, shape=domain.shape, **kwargs)
        return Field(domain, arr)

    def __reduce__(self):
        # host values on the wire, the receiving process's device on arrival
        # (a MAP mean broadcast to ranks that each own a GPU)
        return (Field.from_raw, (self._domain, self.val_np()))

    def __deepcopy__(self, memo):
        return Field(self._domain, self._val.clone())

    # ------------------------------------------------------------ properties
    @property
    def val(self):
        return self._val

    def val_rw(self):
        return self._val.clone()

    def val_np(self):
        return self._val.detach().cpu().numpy()

    def __array__(self, dtype=None, copy=None):
        a = self.val_np()
        return a if dtype is None else a.astype(dtype)

    @property
    def dtype(self):
        return self._val.dtype

    @property
    def domain(self):
        return self._domain

    @property
    def shape(self):
        return self._domain.shape

    @property
    def size(self):
        return self._domain.size

    @property
    def real(self):
        return Field(self._domain, self._val.real.contiguous() if self._val.is_complex() else self._val)

    @property
    def imag(self):
        if not self._val.is_complex():
            return Field(self._domain, torch.zeros_like(self._val))
        return Field(self._domain, self._val.imag.contiguous())

    def scalar_weight(self, spaces=None):
        return self._domain.scalar_weight(spaces)

    def total_volume(self, spaces=None):
        return self._domain.total_volume(spaces)

    def weight(self, power=1, spaces=None):
        aout = self._val
        spaces = utilities.parse_spaces(spaces, len(self._domain))
        fct = 1.
        for ind in spaces:
            wgt = self._domain[ind].dvol
            if np.isscalar(wgt):
                fct *= wgt
            else:
                new_shape = np.ones(len(self.shape), dtype=np.int64)
                new_shape[self._domain.axes[ind][0]:self._domain.axes[ind][-1] + 1] = np.shape(wgt)
                w = torch.as_tensor(np.asarray(wgt) ** power, device=aout.device, dtype=aout.dtype)
                aout = aout * w.reshape(tuple(new_shape))
        if fct != 1.:
            aout = aout * (fct ** power)
        return Field(self._domain, aout)

    # ------------------------------------------------------------ reductions
    def vdot(self, x, spaces=None):
        from .ducc_dispatch import vdot
        if not isinstance(x, Field):
            raise TypeError("The dot-partner must be an instance of the Field class")
        utilities.check_object_identity(x._domain, self._domain)
        ndom = len(self._domain)
        spaces = utilities.parse_spaces(spaces, ndom)
        if len(spaces) == ndom:
            return Field.scalar(vdot(self._val, x._val))
        return (self.conjugate() * x).sum(spaces=spaces)

    def s_vdot(self, x):
        """Python scalar sum(conj(self)*x) (synchronises; fused solvers avoid it)."""
        from .ducc_dispatch import vdot
        if not isinstance(x, Field):
            raise TypeError("The dot-partner must be an instance of the Field class")
        utilities.check_object_identity(x._domain, self._domain)
        return vdot(self._val, x._val).item()

    def norm(self, ord=2):
        if ord == 2:
            from .ducc_dispatch import vdot
            v = self._val
            if v.is_complex():
                v = torch.view_as_real(v).reshape(-1).contiguous()
            return float(np.sqrt(max(vdot(v, v).item(), 0.)))
        return float(torch.linalg.vector_norm(self._val.reshape(-1), ord=ord).item())

    def conjugate(self):
        return Field(self._domain, self._val.conj().resolve_conj()) if self._val.is_complex() else self

    def __pos__(self):
        return self

    def __neg__(self):
        return Field(self._domain, -self._val)

    def __abs__(self):
        return Field(self._domain, torch.abs(self._val))

    def _contraction_helper(self, op, spaces):
        if spaces is None:
            return Field.scalar(getattr(torch, op)(self._val))
        spaces = utilities.parse_spaces(spaces, len(self._domain))
        axes_list = tuple(self._domain.axes[sp_index] for sp_index in spaces)
        axes_list = tuple(a for ax in axes_list for a in ax)
        data = self._val
        if len(axes_list) > 0:
            data = getattr(torch, op)(data, dim=axes_list) if op != "prod" else _prod_axes(data, axes_list)
        return_domain = tuple(dom for i, dom in enumerate(self._domain) if i not in spaces)
        return Field(DomainTuple.make(return_domain), data)

    def sum(self, spaces=None):
        return self._contraction_helper("sum", spaces)

    def s_sum(self):
        return self._val.sum().item()

    def integrate(self, spaces=None):
        swgt = self.scalar_weight(spaces)
        if swgt is not None:
            res = self.sum(spaces)
            return res * swgt
        return self.weight(1, spaces=spaces).sum(spaces)

    def s_integrate(self):
        swgt = self.scalar_weight()
        if swgt is not None:
            return self.s_sum() * swgt
        return self.weight(1).s_sum()

    def prod(self, spaces=None):
        return self._contraction_helper("prod", spaces)

    def s_prod(self):
        return self._val.prod().item()

    def all(self, spaces=None):
        return self._contraction_helper("all", spaces)

    def s_all(self):
        return bool(self._val.all().item())

    def any(self, spaces=None):
        return self._contraction_helper("any", spaces)

    def s_any(self):
        return bool(self._val.any().item())

    def mean(self, spaces=None):
        if self.scalar_weight(spaces) is not None:
            return self._contraction_helper("mean", spaces)
        return self.integrate(spaces) / self.total_volume(spaces)

    def s_mean(self):
        return self.mean().val.item()

    def __repr__(self):
        return "<nifty_amd.Field>"

    def __str__(self):
        return f"nifty_amd.Field instance\n- domain = {self._domain}\n- val    = {self._val!r}"

    def extract(self, dom):
        utilities.check_object_identity(dom, self._domain)
        return self

    def extract_part(self, dom):
        utilities.check_object_identity(dom, self._domain)
        return self

    def unite(self, other):
        return self + other

    def flexible_addsub(self, other, neg):
        return self - other if neg else self + other

    def _binary_op(self, other, op):
        if isinstance(other, Field):
            utilities.check_object_identity(other._domain, self._domain)
            return Field(self._domain, _OPS[op](self._val, other._val))
        if np.isscalar(other) or (isinstance(other, torch.Tensor) and other.ndim == 0):
            return Field(self._domain, _OPS[op](self._val, other))
        return NotImplemented

    def ptw(self, op, *args, **kwargs):
        from .pointwise import ptw_dict
        return Field(self._domain, ptw_dict[op][0](self._val, *args, **kwargs))

    def ptw_with_deriv(self, op, *args, **kwargs):
        from .pointwise import ptw_dict
        tmp = ptw_dict[op][1](self._val, *args, **kwargs)
        return Field(self._domain, tmp[0]), Field(self._domain, tmp[1])

    def clip(self, a_min=None, a_max=None):
        return Field(self._domain, torch.clip(self._val, a_min, a_max))

    def outer(self, x):
        if not isinstance(x, Field):
            raise TypeError
        return Field(DomainTuple.make(tuple(self._domain) + tuple(x._domain)),
                     torch.tensordot(self._val, x._val, dims=0))

    def __bool__(self):
        raise TypeError("Field does not support implicit conversion to bool")


def _prod_axes(data, axes):
    for a in sorted(axes, reverse=True):
        data = torch.prod(data, dim=a)
    return data


_OPS = {
    "__add__": lambda a, b: a + b, "__radd__": lambda a, b: b + a,
    "__sub__": lambda a, b: a - b, "__rsub__": lambda a, b: b - a,
    "__mul__": lambda a, b: a * b, "__rmul__": lambda a, b: b * a,
    "__truediv__": lambda a, b: a / b, "__rtruediv__": lambda a, b: b / a,
    "__floordiv__": lambda a, b: a // b, "__rfloordiv__": lambda a, b: b // a,
    "__pow__": lambda a, b: a ** b, "__rpow__": lambda a, b: b ** a,
    "__lt__": lambda a, b: a < b, "__le__": lambda a, b: a <= b,
    "__gt__": lambda a, b: a > b, "__ge__": lambda a, b: a >= b,
    "__eq__": lambda a, b: a == b, "__ne__": lambda a, b: a != b,
    "__and__": lambda a, b: a & b, "__or__": lambda a, b: a | b,
}


def _mkop(op):
    def f(self, other):
        return self._binary_op(other, op)
    return f


for _op in _OPS:
    setattr(Field, _op, _mkop(_op))
Field.__hash__ = None

for _f in ("sqrt", "exp", "log", "sin", "cos", "tan", "sinh", "cosh", "tanh", "sinc", "absolute",
           "sigmoid", "reciprocal", "log10", "log1p", "expm1", "softplus", "arctan", "sign"):
    setattr(Field, _f, (lambda name: lambda self: self.ptw(name))(_f))

# duck-typing hooks shared with Operator/Linearization (a Field is a constant:
# no Jacobian, no metric)
Field.jac = None
Field.want_metric = False
Field.metric = None
