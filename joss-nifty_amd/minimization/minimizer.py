"""Minimizer protocol (src/minimization/minimizer.py): __call__(energy) -> (energy, status)."""


class Minimizer:
    def __call__(self, energy, preconditioner=None):
        raise NotImplementedError
