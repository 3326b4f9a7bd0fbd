"""EndomorphicOperator (src/operators/endomorphic_operator.py:24-81)."""
from ..utilities import check_object_identity
from .linear_operator import LinearOperator


class EndomorphicOperator(LinearOperator):
    @property
    def target(self):
        return self._domain

    def draw_sample(self, from_inverse=False):
        raise NotImplementedError

    @property
    def sampling_dtype(self):
        return getattr(self, "_dtype", None)

    def get_sqrt(self):
        raise NotImplementedError

    def _dom(self, mode):
        return self._domain

    def _tgt(self, mode):
        return self._domain

    def _check_input(self, x, mode):
        self._check_mode(mode)
        if self.domain != x.domain:
            raise ValueError("The operator's and field's domains don't match.")
