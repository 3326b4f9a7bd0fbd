"""ContractionOperator (src/operators/contraction_operator.py:28-103)."""
import torch

from .. import utilities
from ..domain_tuple import DomainTuple
from ..field import Field
from .linear_operator import LinearOperator


class ContractionOperator(LinearOperator):
    def __init__(self, domain, spaces, power=0):
        self._domain = DomainTuple.make(domain)
        self._spaces = utilities.parse_spaces(spaces, len(self._domain))
        self._target = DomainTuple.make([d for i, d in enumerate(self._domain) if i not in self._spaces])
        self._power = power
        self._capability = self.TIMES | self.ADJOINT_TIMES

    def apply(self, x, mode):
        self._check_input(x, mode)
        if mode == self.ADJOINT_TIMES:
            shp = []
            for i, dom in enumerate(self._domain):
                shp += list(dom.shape) if i not in self._spaces else [1] * len(dom.shape)
            ldat = x.val.reshape(shp).expand(self._domain.shape)
            res = Field(self._domain, ldat)
            if self._power != 0:
                res = res.weight(self._power, spaces=self._spaces)
            return res
        if self._power != 0:
            x = x.weight(self._power, spaces=self._spaces)
        res = x.sum(self._spaces)
        return res if isinstance(res, Field) else Field.scalar(res)


def IntegrationOperator(domain, spaces):
    return ContractionOperator(domain, spaces, 1)
