"""LinearOperator: mode-based linear maps (src/operators/linear_operator.py).

Modes: TIMES=1, ADJOINT_TIMES=2, INVERSE_TIMES=4, ADJOINT_INVERSE_TIMES=8.
``apply(x, mode)`` raises NotImplementedError for an unsupported mode and
ValueError for a domain mismatch, as in the reference (:146-168, :247-256)."""
from ..utilities import check_object_identity
from .operator import Operator


class LinearOperator(Operator):
    TIMES = 1
    ADJOINT_TIMES = 2
    INVERSE_TIMES = 4
    ADJOINT_INVERSE_TIMES = 8
    INVERSE_ADJOINT_TIMES = 8
    ADJOINT_BIT = 1
    INVERSE_BIT = 2
    _ilog = (-1, 0, 1, -1, 2, -1, -1, -1, 3)
    _validMode = (False, True, True, False, True, False, False, False, True)
    _modeTable = ((1, 2, 4, 8), (2, 1, 8, 4), (4, 8, 1, 2), (8, 4, 2, 1))
    _capTable = ((0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15),
                 (0, 2, 1, 3, 8, 10, 9, 11, 4, 6, 5, 7, 12, 14, 13, 15),
                 (0, 4, 8, 12, 1, 5, 9, 13, 2, 6, 10, 14, 3, 7, 11, 15),
                 (0, 8, 4, 12, 2, 10, 6, 14, 1, 9, 5, 13, 3, 11, 7, 15))
    _addInverse = (0, 5, 10, 15, 5, 5, 15, 15, 10, 15, 10, 15, 15, 15, 15, 15)
    _backwards = 6
    _all_ops = 15

    def _dom(self, mode):
        return self.domain if (mode & 9) else self.target

    def _tgt(self, mode):
        return self.domain if (mode & 6) else self.target

    def _flip_modes(self, trafo):
        from .operator_adapter import OperatorAdapter
        return self if trafo == 0 else OperatorAdapter(self, trafo)

    @property
    def inverse(self):
        return self._flip_modes(self.INVERSE_BIT)

    @property
    def adjoint(self):
        return self._flip_modes(self.ADJOINT_BIT)

    def __matmul__(self, other):
        if isinstance(other, LinearOperator):
            from .chain_operator import ChainOperator
            return ChainOperator.make([self, other])
        return Operator.__matmul__(self, other)

    def __rmatmul__(self, other):
        if isinstance(other, LinearOperator):
            from .chain_operator import ChainOperator
            return ChainOperator.make([other, self])
        return Operator.__rmatmul__(self, other)

    def _myadd(self, other, oneg):
        from .sum_operator import SumOperator
        return SumOperator.make((self, other), (False, oneg))

    def __add__(self, other):
        if isinstance(other, LinearOperator):
            return self._myadd(other, False)
        return Operator.__add__(self, other)

    def __radd__(self, other):
        return self.__add__(other)

    def __sub__(self, other):
        if isinstance(other, LinearOperator):
            return self._myadd(other, True)
        return Operator.__sub__(self, other)

    def __rsub__(self, other):
        if isinstance(other, LinearOperator):
            return other._myadd(self, True)
        return NotImplemented

    @property
    def capability(self):
        return self._capability

    def force(self, x):
        return self.apply(x.extract(self.domain), self.TIMES)

    def apply(self, x, mode):
        raise NotImplementedError

    def __call__(self, x):
        from .operator import _is_fieldlike, _is_lin
        if _is_lin(x):
            return x.new(self(x._val), self).prepend_jac(x.jac)
        if _is_fieldlike(x):
            return self.apply(x, self.TIMES)
        return self @ x

    def times(self, x):
        return self.apply(x, self.TIMES)

    def inverse_times(self, x):
        return self.apply(x, self.INVERSE_TIMES)

    def adjoint_times(self, x):
        return self.apply(x, self.ADJOINT_TIMES)

    def adjoint_inverse_times(self, x):
        return self.apply(x, self.ADJOINT_INVERSE_TIMES)

    def inverse_adjoint_times(self, x):
        return self.apply(x, self.ADJOINT_INVERSE_TIMES)

    def _check_mode(self, mode):
        if not self._validMode[mode]:
            raise NotImplementedError("invalid operator mode specified")
        if mode & self.capability == 0:
            raise NotImplementedError("requested operator mode is not supported")

    def _check_input(self, x, mode):
        self._check_mode(mode)
        check_object_identity(self._dom(mode), x.domain)
