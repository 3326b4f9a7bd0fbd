"""ScalingOperator (src/operators/scaling_operator.py:24-130)."""
import numpy as np

from .endomorphic_operator import EndomorphicOperator


class ScalingOperator(EndomorphicOperator):
    def __init__(self, domain, factor, sampling_dtype=None):
        from ..sugar import makeDomain
        if not np.isscalar(factor):
            raise TypeError("Scalar required")
        self._domain = makeDomain(domain)
        self._factor = factor
        self._capability = self._all_ops
        self._dtype = sampling_dtype

    def apply(self, x, mode):
        from ..sugar import full
        self._check_input(x, mode)
        fct = self._factor
        if fct == 1.:
            return x
        if fct == 0.:
            return full(x.domain, 0.)
        if (mode & (self.ADJOINT_TIMES | self.ADJOINT_INVERSE_TIMES)) != 0:
            fct = np.conj(fct)
        if (mode & (self.INVERSE_TIMES | self.ADJOINT_INVERSE_TIMES)) != 0:
            fct = 1. / fct
        return x * fct

    def _flip_modes(self, trafo):
        fct = self._factor
        if trafo & self.ADJOINT_BIT:
            fct = np.conj(fct)
        if trafo & self.INVERSE_BIT:
            fct = 1. / fct
        return ScalingOperator(self._domain, fct, self._dtype)

    def _get_fct(self, from_inverse):
        fct = self._factor
        if (np.imag(fct) != 0. or np.real(fct) < 0. or (np.real(fct) == 0. and from_inverse)):
            raise ValueError("operator not positive definite")
        return 1. / np.sqrt(fct) if from_inverse else np.sqrt(fct)

    def draw_sample(self, from_inverse=False):
        from ..sugar import from_random
        if self._dtype is None:
            raise RuntimeError("Need to specify dtype to be able to sample from this operator:\n"
                               + repr(self))
        return from_random(domain=self._domain, random_type="normal", dtype=self._dtype,
                           std=self._get_fct(from_inverse))

    def get_sqrt(self):
        fct = self._get_fct(False)
        return ScalingOperator(self._domain, fct, self._dtype)

    def __call__(self, x):
        return super().__call__(x)

    def __repr__(self):
        return f"ScalingOperator ({self._factor})"
