"""Probing helpers for the napprox preconditioner (src/probing.py:24-152).

``approximation2endo(op, n)`` estimates the diagonal of the sampling metric
from ``n`` draws of ``op.draw_sample()`` (samples WITH the metric as
covariance) by their unbiased variance; zero entries become 1.  draw_samples
uses its inverse as the CG preconditioner (kl_energies.py:127-128)."""
import torch

from .field import Field
from .multi_field import MultiField


class StatCalculator:
    """Running mean and unbiased variance (Welford), probing.py:24-71 --
    same update order as the reference."""

    def __init__(self):
        self._count = 0

    def add(self, value):
        self._count += 1
        if self._count == 1:
            self._mean = 1. * value
            self._M2 = 0. * value
        else:
            delta = value - self._mean
            self._mean = self.mean + delta * (1. / self._count)
            delta2 = value - self._mean
            self._M2 = self._M2 + delta * delta2

    @property
    def mean(self):
        if self._count == 0:
            raise RuntimeError
        return 1. * self._mean

    @property
    def var(self):
        if self._count < 2:
            raise RuntimeError
        return self._M2 * (1. / (self._count - 1))


def probe_diagonal(op, nprobes, random_type="pm1"):
    """Mean of conj(v_i) * op(v_i) over random probes (probing.py:112-139)."""
    from .sugar import from_random
    sc = StatCalculator()
    for _ in range(nprobes):
        x = from_random(op.domain, random_type)
        sc.add(op(x).conjugate() * x)
    return sc.mean


def _ones_for_zeros(f):
    v = f.val
    return Field(f.domain, torch.where(v == 0, torch.ones_like(v), v))


def approximation2endo(op, nsamples):
    """probing.py:142-152"""
    sc = StatCalculator()
    for _ in range(nsamples):
        sc.add(op.draw_sample())
    approx = sc.var
    if isinstance(approx, MultiField):
        return MultiField.from_dict({kk: _ones_for_zeros(vv) for kk, vv in approx.items()})
    return _ones_for_zeros(approx)
