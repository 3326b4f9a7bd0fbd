"""Operator base class and its nonlinear combinators (src/operators/operator.py).

Semantics follow the reference: ``op(x)`` for a Field/MultiField evaluates the
operator, ``op(Linearization)`` additionally propagates the Jacobian (forward
mode), ``@`` chains, ``+`` sums, ``*`` multiplies pointwise, ``ptw`` applies a
pointwise function.  Evaluation runs on device tensors."""
import numbers
from functools import reduce

import numpy as np

from ..domain_tuple import DomainTuple
from ..multi_domain import MultiDomain
from ..utilities import check_object_identity, indent


def _is_fieldlike(x):
    from ..field import Field
    from ..multi_field import MultiField
    return isinstance(x, (Field, MultiField))


def _is_lin(x):
    from ..linearization import Linearization
    return isinstance(x, Linearization)


class Operator:
    """Transforms values defined on `domain` into values defined on `target`."""
    _domain = None
    _target = None

    @property
    def domain(self):
        return self._domain

    @property
    def target(self):
        return self._target

    @property
    def val(self):
        return None

    @property
    def jac(self):
        return None

    @property
    def want_metric(self):
        return False

    @property
    def metric(self):
        return None

    def scale(self, factor):
        if not isinstance(factor, numbers.Number):
            raise TypeError(".scale() takes a number as input")
        if factor == 1:
            return self
        from .scaling_operator import ScalingOperator
        return ScalingOperator(self.target, factor)(self)

    def conjugate(self):
        from .simple_linear_operators import ConjugationOperator
        return ConjugationOperator(self.target)(self)

    def sum(self, spaces=None):
        from .contraction_operator import ContractionOperator
        return ContractionOperator(self.target, spaces)(self)

    def integrate(self, spaces=None):
        from .contraction_operator import IntegrationOperator
        return IntegrationOperator(self.target, spaces)(self)

    def power(self, exponent):
        return self.ptw("power", exponent)

    def vdot(self, other):
        from ..sugar import makeOp
        if other.jac is None and _is_fieldlike(other):
            res = self.conjugate() * other
        else:
            res = makeOp(other) @ self.conjugate()
        return res.sum()

    @property
    def real(self):
        from .simple_linear_operators import Realizer
        return Realizer(self.target)(self)

    def __neg__(self):
        return self.scale(-1)

    def __matmul__(self, x):
        from .energy_operators import LikelihoodEnergyOperator
        if not isinstance(x, Operator) or isinstance(x, LikelihoodEnergyOperator):
            return NotImplemented
        if x.target is self.domain:
            return _OpChain.make((self, x))
        return self.partial_insert(x)

    def __rmatmul__(self, x):
        from .energy_operators import LikelihoodEnergyOperator
        if not isinstance(x, Operator) or isinstance(x, LikelihoodEnergyOperator):
            return NotImplemented
        if x.domain is self.target:
            return _OpChain.make((x, self))
        return x.partial_insert(self)

    def partial_insert(self, x):
        if not isinstance(self.domain, MultiDomain) or not isinstance(x.target, MultiDomain):
            raise TypeError("partial insertion needs MultiDomains")
        bigdom = MultiDomain.union([self.domain, x.target])
        k1, k2 = set(self.domain.keys()), set(x.target.keys())
        le, ri = k2 - k1, k1 - k2
        leop, riop = self, x
        if len(ri) > 0:
            riop = riop + self.identity_operator(MultiDomain.make({kk: bigdom[kk] for kk in ri}))
        if len(le) > 0:
            leop = leop + self.identity_operator(MultiDomain.make({kk: bigdom[kk] for kk in le}))
        return leop @ riop

    @staticmethod
    def identity_operator(dom):
        from ..sugar import makeDomain
        from .block_diagonal_operator import BlockDiagonalOperator
        from .scaling_operator import ScalingOperator
        dom = makeDomain(dom)
        if isinstance(dom, DomainTuple):
            return ScalingOperator(dom, 1.)
        return BlockDiagonalOperator(dom, {kk: ScalingOperator(dd, 1.) for kk, dd in dom.items()})

    def __mul__(self, x):
        if isinstance(x, Operator):
            return _OpProd(self, x)
        if np.isscalar(x):
            return self.scale(x)
        return NotImplemented

    def __rmul__(self, x):
        return self.__mul__(x)

    def __add__(self, x):
        if not isinstance(x, Operator):
            return NotImplemented
        return _OpSum(self, x)

    def __sub__(self, x):
        if not isinstance(x, Operator):
            return NotImplemented
        return _OpSum(self, -x)

    def __abs__(self):
        return self.ptw("abs")

    def __pow__(self, power):
        if not np.isscalar(power):
            return NotImplemented
        return self.ptw("power", power)

    def __getitem__(self, key):
        from .simple_linear_operators import ducktape
        if not isinstance(self.target, MultiDomain):
            raise TypeError("Only Operators with a MultiDomain as target can be subscripted.")
        return ducktape(None, self, key) @ self

    def apply(self, x):
        raise NotImplementedError

    def force(self, x):
        return self.apply(x.extract(self.domain))

    def _check_input(self, x):
        from .scaling_operator import ScalingOperator
        if not (_is_fieldlike(x) or _is_lin(x)):
            raise TypeError(f"cannot apply operator to {type(x)}")
        if x.jac is not None:
            if not isinstance(x.jac, ScalingOperator) or x.jac._factor != 1:
                raise ValueError("input Linearization must have an identity Jacobian")
        check_object_identity(self._domain, x.domain)

    def __call__(self, x):
        """(operator.py:294-301): Linearization -> chain rule via prepend_jac,
        Field -> evaluation, Operator -> composition."""
        if _is_lin(x):
            return self.apply(x.trivial_jac()).prepend_jac(x.jac)
        if _is_fieldlike(x):
            return self.apply(x)
        if isinstance(x, Operator):
            return self @ x
        raise TypeError(f"cannot apply operator to {type(x)}")

    def ducktape(self, name):
        from .simple_linear_operators import ducktape
        return self @ ducktape(self, None, name)

    def ducktape_left(self, name):
        from .simple_linear_operators import ducktape
        return ducktape(None, self, name) @ self

    def __repr__(self):
        return self.__class__.__name__

    def simplify_for_constant_input(self, c_inp):
        from ..multi_field import MultiField
        if c_inp is None or (isinstance(c_inp, MultiField) and len(c_inp.keys()) == 0):
            return None, self
        if isinstance(c_inp.domain, MultiDomain) and len(c_inp.domain) == 0:
            return None, self
        if isinstance(self.domain, MultiDomain) and isinstance(c_inp.domain, MultiDomain):
            if not set(c_inp.keys()) <= set(self.domain.keys()):
                raise ValueError("constant keys are not a subset of the operator's domain")
        if c_inp.domain == self.domain:
            op = _ConstantOperator(self.force(c_inp))
            return op(c_inp), op
        if not isinstance(c_inp.domain, MultiDomain):
            raise RuntimeError
        return self._simplify_for_constant_input_nontrivial(c_inp)

    def _simplify_for_constant_input_nontrivial(self, c_inp):
        from .simplify_for_const import InsertionOperator
        return None, self @ InsertionOperator(self.domain, c_inp)

    def ptw(self, op, *args, **kwargs):
        return _OpChain.make((_FunctionApplier(self.target, op, *args, **kwargs), self))

    def ptw_pre(self, op, *args, **kwargs):
        return _OpChain.make((self, _FunctionApplier(self.domain, op, *args, **kwargs)))


def _is_identity_lin(x):
    from .scaling_operator import ScalingOperator
    return isinstance(x.jac, ScalingOperator) and x.jac._factor == 1


for _f in ["sqrt", "exp", "log", "sin", "cos", "tan", "sinh", "cosh", "tanh", "sinc", "sigmoid",
           "absolute", "reciprocal", "log10", "log1p", "expm1", "softplus", "arctan", "one_over"]:
    _name = "reciprocal" if _f == "one_over" else _f
    setattr(Operator, _f, (lambda name: lambda self: self.ptw(name))(_name))


class _ConstantOperator(Operator):
    def __init__(self, output, domain=None):
        from ..sugar import makeDomain
        self._domain = makeDomain({}) if domain is None else domain
        self._target = output.domain
        self._output = output

    def apply(self, x):
        from ..linearization import Linearization
        from .simple_linear_operators import NullOperator
        if _is_lin(x):
            return x.new(self._output, NullOperator(x.domain, self._target))
        return self._output

    def __call__(self, x):
        return self.apply(x)


class _FunctionApplier(Operator):
    def __init__(self, domain, funcname, *args, **kwargs):
        from ..sugar import makeDomain
        self._domain = self._target = makeDomain(domain)
        self._funcname = funcname
        self._args = args
        self._kwargs = kwargs

    def apply(self, x):
        self._check_input(x)
        return x.ptw(self._funcname, *self._args, **self._kwargs)

    def __repr__(self):
        return f"_FunctionApplier ('{self._funcname}')"


class _CombinedOperator(Operator):
    def __init__(self, ops, _callingfrommake=False):
        if not _callingfrommake:
            raise NotImplementedError
        self._ops = tuple(ops)

    @classmethod
    def unpack(cls, ops, res):
        for op in ops:
            if isinstance(op, cls):
                res = cls.unpack(op._ops, res)
            else:
                res = res + [op]
        return res

    @classmethod
    def make(cls, ops):
        res = cls.unpack(ops, [])
        if len(res) == 1:
            return res[0]
        return cls(res, _callingfrommake=True)


class _OpChain(_CombinedOperator):
    def __init__(self, ops, _callingfrommake=False):
        super().__init__(ops, _callingfrommake)
        self._domain = self._ops[-1].domain
        self._target = self._ops[0].target
        for i in range(1, len(self._ops)):
            check_object_identity(self._ops[i - 1].domain, self._ops[i].target)

    def apply(self, x):
        self._check_input(x)
        for op in reversed(self._ops):
            x = op(x)
        return x

    def _simplify_for_constant_input_nontrivial(self, c_inp):
        if not isinstance(self._domain, MultiDomain):
            return None, self
        newop = None
        for op in reversed(self._ops):
            c_inp, t_op = op.simplify_for_constant_input(c_inp)
            newop = t_op if newop is None else op(newop)
        return c_inp, newop

    def __repr__(self):
        return "_OpChain:\n" + indent("\n".join(repr(s) for s in self._ops))


class _OpProd(Operator):
    def __init__(self, op1, op2):
        from ..sugar import domain_union
        self._domain = domain_union((op1.domain, op2.domain))
        self._target = op1.target
        if op1.target != op2.target:
            raise ValueError("target mismatch")
        self._op1, self._op2 = op1, op2

    def apply(self, x):
        from ..linearization import Linearization
        from ..sugar import makeOp
        self._check_input(x)
        lin = x.jac is not None
        wm = x.want_metric if lin else False
        x = x.val if lin else x
        v1 = x.extract(self._op1.domain)
        v2 = x.extract(self._op2.domain)
        if not lin:
            return self._op1(v1) * self._op2(v2)
        lin1 = self._op1(Linearization.make_var(v1, wm))
        lin2 = self._op2(Linearization.make_var(v2, wm))
        jac = (makeOp(lin1._val)(lin2._jac))._myadd(makeOp(lin2._val)(lin1._jac), False)
        return lin1.new(lin1._val * lin2._val, jac)

    def __repr__(self):
        return "_OpProd:\n" + indent("\n".join(repr(s) for s in (self._op1, self._op2)))


class _OpSum(Operator):
    def __init__(self, op1, op2):
        from ..sugar import domain_union
        self._domain = domain_union((op1.domain, op2.domain))
        self._target = domain_union((op1.target, op2.target))
        self._op1, self._op2 = op1, op2

    def apply(self, x):
        from ..linearization import Linearization
        self._check_input(x)
        ops = [self._op1, self._op2]
        unite = lambda a, b: a.unite(b)  # noqa: E731
        if x.jac is None:
            return reduce(unite, (oo.force(x) for oo in ops))
        lin = [oo(Linearization.make_var(x.val.extract(oo.domain), x.want_metric)) for oo in ops]
        jac = reduce(lambda a, b: a._myadd(b, False), (ll._jac for ll in lin))
        val = reduce(unite, (ll._val for ll in lin))
        res = x.new(val, jac)
        metrics = [ll._metric for ll in lin]
        if all(mm is not None for mm in metrics):
            res = res.add_metric(reduce(lambda a, b: a + b, metrics))
        return res

    def __repr__(self):
        return "_OpSum:\n" + indent("\n".join(repr(s) for s in (self._op1, self._op2)))
