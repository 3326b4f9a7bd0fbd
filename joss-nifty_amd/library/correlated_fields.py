"""Correlated-field amplitude building blocks
(src/library/correlated_fields.py:43-212).

The linear helpers (_SlopeRemover, _TwoLogIntegrations, _SpecialSum) are
provided as LinearOperators for API parity, and the same math is exposed as
plain tensor functions (``twolog``, ``twolog_adjoint``, ``slope_remove``...)
used by the fused amplitude model of correlated_fields_simple.py.  All of it
works on B-sized power-spectrum arrays (B = number of |k| bins), i.e. a small
fraction of the grid."""
import numpy as np
import torch

from ..domain_tuple import DomainTuple
from ..domains import PowerSpace, UnstructuredDomain
from ..field import Field
from ..operators.endomorphic_operator import EndomorphicOperator
from ..operators.linear_operator import LinearOperator
from ..sugar import makeDomain
from ..utilities import myassert


def _log_k_lengths(pspace):
    """log(k_lengths) without zeromode (correlated_fields.py:50-52)"""
    return np.log(pspace.k_lengths[1:])


def _relative_log_k_lengths(power_space):
    """log-distance to the first bin; [0]=[1]=0 (:55-64)"""
    if isinstance(power_space, DomainTuple):
        power_space = power_space[0]
    logkl = _log_k_lengths(power_space)
    logkl = logkl - logkl[0]
    return np.insert(logkl, 0, 0)


def _log_vol(power_space):
    """(:67-71)"""
    if isinstance(power_space, DomainTuple):
        power_space = power_space[0]
    logk = _log_k_lengths(power_space)
    return logk[1:] - logk[:-1]


# --------------------------------------------------------------- tensor math
def twolog(x0, x1, lv):
    """_TwoLogIntegrations TIMES on (2, B-2) -> (B,) (:127-143)."""
    c = torch.cumsum(x1, 0)
    cprev = torch.cat([c.new_zeros(1), c[:-1]])
    t = (c + cprev) / 2 * lv + x0
    return torch.cat([c.new_zeros(2), torch.cumsum(t, 0)])


def _revcumsum(v):
    return torch.flip(torch.cumsum(torch.flip(v, (0,)), 0), (0,))


def twolog_adjoint(g, lv):
    """_TwoLogIntegrations ADJOINT_TIMES on (B,) -> ((B-2,), (B-2,)) (:144-155)."""
    y = _revcumsum(g[2:])
    z = y * (lv / 2.)
    w = z + torch.cat([z[1:], z.new_zeros(1)])
    return y, _revcumsum(w)


def slope_remove(x, sc):
    """_SlopeRemover TIMES (:105-110)"""
    return x - x[-1] * sc


def slope_remove_adjoint(x, sc):
    """_SlopeRemover ADJOINT (:111-113)"""
    res = x.clone()
    res[-1] = res[-1] - torch.sum(x * sc)
    return res


# --------------------------------------------------------------- operators
def _dev_tensor(a):
    from .. import config
    return torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float64, device=config.device())


class _SlopeRemover(EndomorphicOperator):
    def __init__(self, domain, space=0):
        self._domain = makeDomain(domain)
        myassert(isinstance(self._domain[space], PowerSpace))
        if len(self._domain) != 1:
            raise NotImplementedError("only single-space power domains are supported")
        logkl = _relative_log_k_lengths(self._domain[space])
        self._sc = _dev_tensor(logkl / float(logkl[-1]))
        self._capability = self.TIMES | self.ADJOINT_TIMES

    def apply(self, x, mode):
        self._check_input(x, mode)
        if mode == self.TIMES:
            return Field(self._domain, slope_remove(x.val, self._sc))
        return Field(self._domain, slope_remove_adjoint(x.val, self._sc))


class _TwoLogIntegrations(LinearOperator):
    def __init__(self, target, space=0):
        self._target = makeDomain(target)
        myassert(isinstance(self.target[space], PowerSpace))
        if len(self._target) != 1:
            raise NotImplementedError("only single-space power domains are supported")
        self._domain = makeDomain(UnstructuredDomain((2, self.target[space].shape[0] - 2)))
        self._lv = _dev_tensor(_log_vol(self._target[space]))
        self._capability = self.TIMES | self.ADJOINT_TIMES

    def apply(self, x, mode):
        self._check_input(x, mode)
        if mode == self.TIMES:
            v = x.val
            return Field(self._target, twolog(v[0], v[1], self._lv))
        r0, r1 = twolog_adjoint(x.val, self._lv)
        return Field(self._domain, torch.stack([r0, r1]))


class _SpecialSum(EndomorphicOperator):
    def __init__(self, domain, space=0):
        self._domain = makeDomain(domain)
        self._capability = self.TIMES | self.ADJOINT_TIMES

    def apply(self, x, mode):
        self._check_input(x, mode)
        return Field(self._domain, torch.sum(x.val).expand(self._domain.shape).clone())


def mode_multiplicity(pspace):
    """pd.adjoint(full(1)) with the zero mode set to 0 (_Normalization :171-175)."""
    m = np.bincount(pspace.pindex.ravel(), minlength=pspace.shape[0]).astype(np.float64)
    m[0] = 0.
    return m
