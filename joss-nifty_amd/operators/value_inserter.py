"""ValueInserter (src/operators/value_inserter.py:24-60)."""
import torch

from ..domain_tuple import DomainTuple
from ..field import Field
from .linear_operator import LinearOperator


class ValueInserter(LinearOperator):
    def __init__(self, target, index):
        self._domain = DomainTuple.scalar_domain()
        self._target = DomainTuple.make(target)
        index = tuple(index)
        if not all(isinstance(n, int) and 0 <= n < self.target.shape[i] for i, n in enumerate(index)):
            raise TypeError
        if not len(index) == len(self.target.shape):
            raise ValueError
        self._index = index
        self._capability = self.TIMES | self.ADJOINT_TIMES

    def apply(self, x, mode):
        self._check_input(x, mode)
        v = x.val
        if mode == self.TIMES:
            res = torch.zeros(self.target.shape, dtype=v.dtype, device=v.device)
            res[self._index] = v
            return Field(self._tgt(mode), res)
        return Field.scalar(v[self._index].clone())
