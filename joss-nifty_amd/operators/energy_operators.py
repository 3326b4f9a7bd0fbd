"""Energy operators on the sampling path (src/operators/energy_operators.py):
GaussianEnergy (:478-583), PoissonianEnergy (:586-625), StandardHamiltonian
(:764-831), the likelihood chain (:152-200) and the quadratic forms."""
import numpy as np

from .. import utilities
from ..domain_tuple import DomainTuple
from ..field import Field
from ..linearization import Linearization
from ..multi_domain import MultiDomain
from ..multi_field import MultiField
from ..sugar import makeDomain
from .adder import Adder
from .linear_operator import LinearOperator
from .operator import Operator, _OpChain
from .sampling_enabler import SamplingEnabler
from .sandwich_operator import SandwichOperator
from .scaling_operator import ScalingOperator
from .simple_linear_operators import VdotOperator


class EnergyOperator(Operator):
    _target = DomainTuple.scalar_domain()


class LikelihoodEnergyOperator(EnergyOperator):
    def __init__(self, data_residual, sqrt_data_metric_at):
        self._res = data_residual
        self._sqrt_data_metric_at = sqrt_data_metric_at
        self._name = None

    def normalized_residual(self, x):
        return (self._sqrt_data_metric_at(x) @ self._res).force(x)

    @property
    def data_domain(self):
        return None if self._res is None else self._res.target

    def get_transformation(self):
        raise NotImplementedError

    def __matmul__(self, other):
        return _LikelihoodChain(self, other)

    def __rmatmul__(self, other):
        return _LikelihoodChain(other, self)

    def get_metric_at(self, x):
        dtp, f = self.get_transformation()
        bun = f(Linearization.make_var(x)).jac
        return SandwichOperator.make(bun, sampling_dtype=dtp)

    @property
    def name(self):
        return self._name

    @name.setter
    def name(self, x):
        self._name = x


class _LikelihoodChain(LikelihoodEnergyOperator):
    def __init__(self, op1, op2):
        from .simple_linear_operators import PartialExtractor
        self._op = _OpChain.make((op1, op2))
        self._domain = self._op.domain
        if isinstance(op1, ScalingOperator):
            res = op2._res
            sqrt_data_metric_at = op2._sqrt_data_metric_at
        elif op1._res is None:
            res = None
            sqrt_data_metric_at = None
        else:
            if isinstance(op2.target, MultiDomain):
                extract = PartialExtractor(op2.target, op1._res.domain)
            else:
                extract = Operator.identity_operator(op2.target)
            res = op1._res @ extract @ op2
            sqrt_data_metric_at = lambda x: op1._sqrt_data_metric_at(op2.force(x))  # noqa: E731
        super().__init__(res, sqrt_data_metric_at)
        self.name = (op2 if isinstance(op1, ScalingOperator) else op1).name

    def get_transformation(self):
        scaled_lh = isinstance(self._op._ops[0], ScalingOperator)
        ii = 1 if scaled_lh else 0
        tr = self._op._ops[ii].get_transformation()
        if tr is None:
            return tr
        dtype, trafo = tr
        if scaled_lh:
            trafo = trafo.scale(np.sqrt(self._op._ops[0]._factor))
        return dtype, _OpChain.make((trafo,) + self._op._ops[ii + 1:])

    def apply(self, x):
        self._check_input(x)
        return self._op(x)


class Squared2NormOperator(EnergyOperator):
    def __init__(self, domain):
        self._domain = domain

    def apply(self, x):
        self._check_input(x)
        if x.jac is None:
            return x.vdot(x)
        res = x.val.vdot(x.val)
        return x.new(res, VdotOperator(2 * x.val))


class QuadraticFormOperator(EnergyOperator):
    def __init__(self, endo):
        from .endomorphic_operator import EndomorphicOperator
        if not isinstance(endo, EndomorphicOperator):
            raise TypeError("op must be an EndomorphicOperator")
        self._op = endo
        self._domain = endo.domain

    def apply(self, x):
        self._check_input(x)
        if x.jac is None:
            return 0.5 * x.vdot(self._op(x))
        res = 0.5 * x.val.vdot(self._op(x.val))
        return x.new(res, VdotOperator(self._op(x.val)))


def _field_dtype(f):
    from ..utilities import numpy_dtype
    if isinstance(f, Field):
        return numpy_dtype(f.dtype)
    return {k: numpy_dtype(v.dtype) for k, v in f.items()}


class GaussianEnergy(LikelihoodEnergyOperator):
    """0.5 (f-d)^dagger D^-1 (f-d)."""

    def __init__(self, data=None, inverse_covariance=None, domain=None, sampling_dtype=None):
        if inverse_covariance is not None and not isinstance(inverse_covariance, LinearOperator):
            raise TypeError
        self._domain = self._parseDomain(data, inverse_covariance, domain)
        if not isinstance(data, (Field, MultiField)) and data is not None:
            raise TypeError
        self._icov = inverse_covariance
        if inverse_covariance is None:
            self._op = Squared2NormOperator(self._domain).scale(0.5)
            dt = sampling_dtype if data is None else _field_dtype(data)
            self._icov = ScalingOperator(self._domain, 1., dt)
        else:
            self._op = QuadraticFormOperator(inverse_covariance)
            self._icov = inverse_covariance
        self._data = data
        res = Operator.identity_operator(self._domain) if data is None else Adder(data, neg=True)
        super().__init__(res, lambda x: self.get_metric_at(x).get_sqrt())

    @staticmethod
    def _checkEquivalence(olddom, newdom):
        newdom = makeDomain(newdom)
        if olddom is None:
            return newdom
        utilities.check_object_identity(olddom, newdom)
        return newdom

    def _parseDomain(self, data, inverse_covariance, domain):
        dom = None
        if inverse_covariance is not None:
            dom = self._checkEquivalence(dom, inverse_covariance.domain)
        if data is not None:
            dom = self._checkEquivalence(dom, data.domain)
        if domain is not None:
            dom = self._checkEquivalence(dom, domain)
        if dom is None:
            raise ValueError("no domain given")
        return dom

    def apply(self, x):
        self._check_input(x)
        residual = x if self._data is None else x - self._data
        res = self._op(residual).real
        if x.want_metric:
            return res.add_metric(self.get_metric_at(x.val))
        return res

    def get_transformation(self):
        return self._icov.sampling_dtype, self._icov.get_sqrt()

    def __repr__(self):
        return "GaussianEnergy"


class PoissonianEnergy(LikelihoodEnergyOperator):
    """sum(f) - d^T log(f) for integer counts d."""

    def __init__(self, d):
        if not isinstance(d, Field) or d.dtype not in (np.int64, np.int32, __import__("torch").int64,
                                                        __import__("torch").int32):
            raise TypeError("data is of invalid data-type; counts need to be integers")
        if bool((d.val < 0).any().item()):
            raise ValueError("count data is negative and thus can not be Poissonian")
        self._d = d
        self._dfloat = Field(d.domain, d.val.to(__import__("torch").float64))
        self._domain = DomainTuple.make(d.domain)
        super().__init__(Adder(self._dfloat, neg=True), lambda x: self.get_metric_at(x).get_sqrt())

    def apply(self, x):
        self._check_input(x)
        res = x.sum() - x.log().vdot(self._dfloat)
        if not x.want_metric:
            return res
        return res.add_metric(self.get_metric_at(x.val))

    def get_transformation(self):
        return np.float64, 2. * Operator.identity_operator(self._domain).sqrt()


class StandardHamiltonian(EnergyOperator):
    """0.5 xi^dagger xi + E_lh(xi) (energy_operators.py:764-831)."""

    def __init__(self, lh, ic_samp=None):
        self._lh = lh
        self._prior = GaussianEnergy(data=None, domain=lh.domain, sampling_dtype=float)
        self._ic_samp = ic_samp
        self._domain = lh.domain

    def apply(self, x):
        self._check_input(x)
        lhx, prx = self._lh(x), self._prior(x)
        if not x.want_metric or self._ic_samp is None:
            return lhx + prx
        met = SamplingEnabler(lhx.metric, prx.metric, self._ic_samp)
        return (lhx + prx).add_metric(met)

    @property
    def prior_energy(self):
        return self._prior

    @property
    def likelihood_energy(self):
        return self._lh

    @property
    def iteration_controller(self):
        return self._ic_samp

    def __repr__(self):
        return "StandardHamiltonian:\n" + utilities.indent(repr(self._lh))

    def _simplify_for_constant_input_nontrivial(self, c_inp):
        # energy_operators.py:829-831: the prior of the constant keys is a
        # constant and drops out; the likelihood gets the constants inserted
        out, lh1 = self._lh.simplify_for_constant_input(c_inp)
        return out, StandardHamiltonian(lh1, self._ic_samp)
