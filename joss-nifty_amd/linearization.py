"""Linearization: value + Jacobian (+ metric) of an operator at a point
(src/linearization.py:25-396).  Jacobians are LinearOperator trees whose
leaves run device kernels; fused model operators (e.g. the correlated field)
contribute a single fused Jacobian node."""
import numpy as np

from .operators.operator import Operator
from .utilities import check_object_identity


class Linearization(Operator):
    def __init__(self, val, jac, metric=None, want_metric=False):
        self._val = val
        self._jac = jac
        check_object_identity(self._val.domain, self._jac.target)
        self._want_metric = want_metric
        self._metric = metric

    def new(self, val, jac, metric=None):
        return Linearization(val, jac, metric, self._want_metric)

    def trivial_jac(self):
        return self.make_var(self._val, self._want_metric)

    def prepend_jac(self, jac):
        if self._metric is None:
            return self.new(self._val, self._jac @ jac)
        from .operators.sandwich_operator import SandwichOperator
        metric = SandwichOperator.make(jac, self._metric)
        return self.new(self._val, self._jac @ jac, metric)

    @property
    def domain(self):
        return self._jac.domain

    @property
    def target(self):
        return self._jac.target

    @property
    def val(self):
        return self._val

    @property
    def jac(self):
        return self._jac

    @property
    def gradient(self):
        from .field import Field
        return self._jac.adjoint_times(Field.scalar(1.))

    @property
    def want_metric(self):
        return self._want_metric

    @property
    def metric(self):
        return self._metric

    def __getitem__(self, name):
        return self.new(self._val[name], self._jac.ducktape_left(name))

    def __neg__(self):
        if self._metric is not None:
            raise RuntimeError("Cannot negate operators with metric")
        return self.new(-self._val, -self._jac)

    def conjugate(self):
        return self.new(self._val.conjugate(), self._jac.conjugate(),
                        None if self._metric is None else self._metric.conjugate())

    @property
    def real(self):
        return self.new(self._val.real, self._jac.real)

    def _myadd(self, other, neg):
        if np.isscalar(other) or other.jac is None:
            return self.new(self._val - other if neg else self._val + other, self._jac, self._metric)
        met = None
        if self._metric is not None and other._metric is not None:
            met = self._metric._myadd(other._metric, neg)
        return self.new(self.val.flexible_addsub(other.val, neg), self.jac._myadd(other.jac, neg), met)

    def __add__(self, other):
        return self._myadd(other, False)

    def __radd__(self, other):
        return self._myadd(other, False)

    def __sub__(self, other):
        return self._myadd(other, True)

    def __rsub__(self, other):
        return (-self).__add__(other)

    def __truediv__(self, other):
        if np.isscalar(other):
            return self.__mul__(1 / other)
        return self.__mul__(other.ptw("reciprocal"))

    def __rtruediv__(self, other):
        return self.ptw("reciprocal").__mul__(other)

    def __pow__(self, power):
        if not (np.isscalar(power) or power.jac is None):
            return NotImplemented
        return self.ptw("power", power)

    def __mul__(self, other):
        from .sugar import makeOp
        if np.isscalar(other):
            if other == 1:
                return self
            met = None if self._metric is None else self._metric.scale(other)
            return self.new(self._val * other, self._jac.scale(other), met)
        if other.jac is None:
            check_object_identity(self.target, other.domain)
            return self.new(self._val * other, makeOp(other)(self._jac))
        check_object_identity(self.target, other.target)
        return self.new(self.val * other.val,
                        (makeOp(other.val)(self.jac))._myadd(makeOp(self.val)(other.jac), False))

    def __rmul__(self, other):
        return self.__mul__(other)

    def vdot(self, other):
        from .operators.simple_linear_operators import VdotOperator
        if other.jac is None:
            return self.new(self._val.vdot(other), VdotOperator(other)(self._jac))
        return self.new(self._val.vdot(other._val),
                        VdotOperator(self._val)(other._jac) + VdotOperator(other._val)(self._jac))

    def sum(self, spaces=None):
        from .operators.contraction_operator import ContractionOperator
        return self.new(self._val.sum(spaces), ContractionOperator(self._jac.target, spaces)(self._jac))

    def ptw(self, op, *args, **kwargs):
        from .sugar import makeOp
        t1, t2 = self._val.ptw_with_deriv(op, *args, **kwargs)
        return self.new(t1, makeOp(t2)(self._jac))

    def clip(self, a_min=None, a_max=None):
        return self.ptw("clip", a_min, a_max)

    def add_metric(self, metric):
        return self.new(self._val, self._jac, metric)

    def with_want_metric(self):
        return Linearization(self._val, self._jac, self._metric, True)

    @staticmethod
    def make_var(field, want_metric=False):
        from .operators.scaling_operator import ScalingOperator
        return Linearization(field, ScalingOperator(field.domain, 1.), want_metric=want_metric)

    @staticmethod
    def make_const(field, want_metric=False):
        from .operators.simple_linear_operators import NullOperator
        return Linearization(field, NullOperator(field.domain, field.domain), want_metric=want_metric)

    @staticmethod
    def make_partial_var(field, constants, want_metric=False):
        from .multi_field import MultiField
        from .operators.scaling_operator import ScalingOperator
        from .operators.block_diagonal_operator import BlockDiagonalOperator
        from .operators.simple_linear_operators import NullOperator
        if len(constants) == 0:
            return Linearization.make_var(field, want_metric)
        ops = {kk: (NullOperator(dd, dd) if kk in constants else ScalingOperator(dd, 1.))
               for kk, dd in field.domain.items()}
        return Linearization(field, BlockDiagonalOperator(field.domain, ops), want_metric=want_metric)


for _f in ["sqrt", "exp", "log", "sin", "cos", "tan", "sinh", "cosh", "tanh", "sinc", "sigmoid",
           "absolute", "reciprocal", "log10", "log1p", "expm1", "softplus", "arctan"]:
    setattr(Linearization, _f, (lambda name: lambda self: self.ptw(name))(_f))
