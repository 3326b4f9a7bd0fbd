"""OperatorAdapter: adjoint / inverse views (src/operators/operator_adapter.py)."""
from .linear_operator import LinearOperator


class OperatorAdapter(LinearOperator):
    def __init__(self, op, op_transform):
        self._op = op
        self._trafo = int(op_transform)
        if self._trafo < 1 or self._trafo > 3:
            raise ValueError("invalid operator transformation")
        self._domain = self._op._dom(1 << self._trafo)
        self._target = self._op._tgt(1 << self._trafo)
        self._capability = self._capTable[self._trafo][self._op.capability]

    def _flip_modes(self, trafo):
        newtrafo = trafo ^ self._trafo
        return self._op if newtrafo == 0 else OperatorAdapter(self._op, newtrafo)

    def apply(self, x, mode):
        return self._op.apply(x, self._modeTable[self._trafo][self._ilog[mode]])

    def __repr__(self):
        from ..utilities import indent
        mode = ["adjoint", "inverse", "adjoint inverse"][self._trafo - 1]
        return f"{mode}:\n" + indent(repr(self._op))

    @property
    def wrapped(self):
        return self._op

    @property
    def trafo(self):
        return self._trafo
