"""NormalTransform / LognormalTransform (src/operators/normal_operators.py:24-75)."""
import numpy as np

from ..domain_tuple import DomainTuple
from ..domains import UnstructuredDomain
from ..sugar import makeField
from ..utilities import lognormal_moments, value_reshaper
from .adder import Adder
from .diagonal_operator import DiagonalOperator
from .simple_linear_operators import ducktape


def NormalTransform(mean, sigma, key, N_copies=0):
    if N_copies == 0:
        domain = DomainTuple.scalar_domain()
        mean, sigma = float(mean), float(sigma)
        return Adder(makeField(domain, np.asarray(mean))) @ (sigma * ducktape(domain, None, key))
    domain = DomainTuple.make(UnstructuredDomain(N_copies))
    mean, sigma = (value_reshaper(param, N_copies) for param in (mean, sigma))
    return Adder(makeField(domain, mean)) @ DiagonalOperator(makeField(domain, sigma)) @ ducktape(domain, None, key)


def LognormalTransform(mean, sigma, key, N_copies):
    logmean, logsigma = lognormal_moments(mean, sigma, N_copies)
    return NormalTransform(logmean, logsigma, key, N_copies).ptw("exp")
