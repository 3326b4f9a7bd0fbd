"""FFTOperator / HartleyOperator / HarmonicTransformOperator /
HarmonicSmoothingOperator on RGSpaces (src/operators/harmonic_operators.py:34-423).

The transforms run on the native gfx950 FFT engine through ducc_dispatch
(csrc/nft_fft.hip); volume factors are folded into the final pass."""
import numpy as np

from .. import utilities
from ..domain_tuple import DomainTuple
from ..domains import RGSpace
from ..ducc_dispatch import fftn, hartley, ifftn
from ..field import Field
from .diagonal_operator import DiagonalOperator
from .linear_operator import LinearOperator
from .scaling_operator import ScalingOperator


class FFTOperator(LinearOperator):
    def __init__(self, domain, target=None, space=None):
        self._domain = DomainTuple.make(domain)
        self._capability = self._all_ops
        self._space = utilities.infer_space(self._domain, space)
        adom = self._domain[self._space]
        if not isinstance(adom, RGSpace):
            raise TypeError("FFTOperator only works on RGSpaces")
        if target is None:
            target = adom.get_default_codomain()
        self._target = [dom for dom in self._domain]
        self._target[self._space] = target
        self._target = DomainTuple.make(self._target)
        adom.check_codomain(target)
        target.check_codomain(adom)

    def apply(self, x, mode):
        self._check_input(x, mode)
        ncells = x.domain[self._space].size
        if x.domain[self._space].harmonic:
            func, fct = ifftn, ncells
        else:
            func, fct = fftn, 1.
        axes = x.domain.axes[self._space]
        tdom = self._tgt(mode)
        tmp = func(x.val, axes=axes)
        if mode & (LinearOperator.TIMES | LinearOperator.ADJOINT_TIMES):
            fct *= self._domain[self._space].scalar_dvol
        else:
            fct *= self._target[self._space].scalar_dvol
        return Field(tdom, tmp if fct == 1 else tmp * fct)


class HartleyOperator(LinearOperator):
    def __init__(self, domain, target=None, space=None):
        self._domain = DomainTuple.make(domain)
        self._capability = self._all_ops
        self._space = utilities.infer_space(self._domain, space)
        adom = self._domain[self._space]
        if not isinstance(adom, RGSpace):
            raise TypeError("HartleyOperator only works on RGSpaces")
        if target is None:
            target = adom.get_default_codomain()
        self._target = [dom for dom in self._domain]
        self._target[self._space] = target
        self._target = DomainTuple.make(self._target)
        adom.check_codomain(target)
        target.check_codomain(adom)

    def apply(self, x, mode):
        self._check_input(x, mode)
        if x.val.is_complex():
            return (self._apply_cartesian(x.real, mode) + self._apply_cartesian(x.imag, mode) * 1j)
        return self._apply_cartesian(x, mode)

    def _fct(self, mode):
        if mode & (LinearOperator.TIMES | LinearOperator.ADJOINT_TIMES):
            return self._domain[self._space].scalar_dvol
        return self._target[self._space].scalar_dvol

    def _apply_cartesian(self, x, mode):
        axes = x.domain.axes[self._space]
        tdom = self._tgt(mode)
        # the volume factor is applied inside the last transform pass
        return Field(tdom, hartley(x.val, axes=axes, scale=self._fct(mode)))


class HarmonicTransformOperator(LinearOperator):
    def __init__(self, domain, target=None, space=None):
        domain = DomainTuple.make(domain)
        space = utilities.infer_space(domain, space)
        hspc = domain[space]
        if not hspc.harmonic:
            raise TypeError("HarmonicTransformOperator only works on a harmonic space")
        if not isinstance(hspc, RGSpace):
            raise TypeError("only RGSpace harmonic transforms are supported (SHT is out of scope)")
        self._op = HartleyOperator(domain, target, space)
        self._domain = self._op.domain
        self._target = self._op.target
        self._capability = self.TIMES | self.ADJOINT_TIMES

    def apply(self, x, mode):
        self._check_input(x, mode)
        return self._op.apply(x, mode)


def HarmonicSmoothingOperator(domain, sigma, space=None):
    sigma = float(sigma)
    if sigma < 0.:
        raise ValueError("sigma must be non-negative")
    if sigma == 0.:
        return ScalingOperator(domain, 1.)
    domain = DomainTuple.make(domain)
    space = utilities.infer_space(domain, space)
    if domain[space].harmonic:
        raise TypeError("domain must not be harmonic")
    Hartley = HartleyOperator(domain, space=space)
    codomain = Hartley.domain[space].get_default_codomain()
    kernel = codomain.get_k_length_array()
    smoother = codomain.get_fft_smoothing_kernel_function(sigma)
    kernel = smoother(kernel)
    ddom = list(domain)
    ddom[space] = codomain
    diag = DiagonalOperator(kernel, ddom, space)
    return Hartley.inverse(diag(Hartley))
