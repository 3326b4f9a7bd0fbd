"""QuadraticEnergy: 0.5 x^T A x - b^T x (src/minimization/quadratic_energy.py:27-78)."""
from .energy import Energy


class QuadraticEnergy(Energy):
    def __init__(self, position, A, b, _grad=None):
        super().__init__(position=position)
        self._A = A
        self._b = b
        if _grad is not None:
            self._grad = _grad
            Ax = _grad if b is None else _grad + b
        else:
            Ax = self._A(self._position)
            self._grad = Ax if b is None else Ax - b
        self._value = 0.5 * self._position.s_vdot(Ax).real
        if b is not None:
            self._value -= b.s_vdot(self._position).real

    def at(self, position):
        return QuadraticEnergy(position, self._A, self._b)

    def at_with_grad(self, position, grad):
        return QuadraticEnergy(position, self._A, self._b, grad)

    @property
    def value(self):
        return self._value

    @property
    def gradient(self):
        return self._grad

    @property
    def metric(self):
        return self._A

    def apply_metric(self, x):
        return self._A(x)
