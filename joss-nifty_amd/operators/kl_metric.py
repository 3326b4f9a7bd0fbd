"""Sample-averaged KL metric as an EndomorphicOperator
(SampledKLEnergyClass.metric, src/minimization/kl_energies.py:340-350)."""
from .endomorphic_operator import EndomorphicOperator


class KLMetric(EndomorphicOperator):
    def __init__(self, kl):
        self._kl = kl
        self._domain = kl.position.domain
        self._capability = self.TIMES | self.ADJOINT_TIMES

    def apply(self, x, mode):
        self._check_input(x, mode)
        return self._kl.apply_metric(x)
