"""QuadraticEnergy: 0.5 x^T A x - b^T x (src/minimization/quadratic_energy.py:27-78)."""
from .energy import Energy


class QuadraticEnergy(Energy):
    def __init__(self, position, A, b, _grad=None):
        super().__init__(position=position)
        self._A = A
        self._b = b
        if _grad is not None:
            self._grad = _grad
            self._Ax = None
        else:
            self._Ax = self._A(self._position)
            self._grad = self._Ax if b is None else self._Ax - b
        self._value = None

    def _compute_value(self):
        # evaluated on first use (the same expression, in the same order, as
        # the reference evaluates eagerly): CG and NewtonCG only read the
        # position / gradient of most energies, and each dot is a host sync
        Ax = self._Ax
        if Ax is None:
            Ax = self._grad if self._b is None else self._grad + self._b
        v = 0.5 * self._position.s_vdot(Ax).real
        if self._b is not None:
            v -= self._b.s_vdot(self._position).real
        return v

    def at(self, position):
        return QuadraticEnergy(position, self._A, self._b)

    def at_with_grad(self, position, grad):
        return QuadraticEnergy(position, self._A, self._b, grad)

    @property
    def value(self):
        if self._value is None:
            self._value = self._compute_value()
        return self._value

    @property
    def gradient(self):
        return self._grad

    @property
    def metric(self):
        return self._A

    def apply_metric(self, x):
        return self._A(x)
