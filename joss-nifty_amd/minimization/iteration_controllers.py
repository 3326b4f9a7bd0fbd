"""Iteration controllers (src/minimization/iteration_controllers.py:27-423).
Decisions are taken on host scalars exactly as in the reference, so CG/Newton
iteration counts follow the same rules."""
import functools
import time

import numpy as np

from ..logger import logger
from . import trace as _trace


class IterationController:
    CONVERGED, CONTINUE, ERROR = list(range(3))

    def __init__(self):
        self._history = None

    def start(self, energy):
        raise NotImplementedError

    def check(self, energy):
        raise NotImplementedError

    def enable_logging(self):
        if self._history is None:
            self._history = EnergyHistory()

    def disable_logging(self):
        self._history = None

    @property
    def history(self):
        return self._history


class EnergyHistory:
    def __init__(self):
        self._lst = []

    def append(self, x):
        if len(x) != 2:
            raise ValueError
        self._lst.append((float(x[0]), float(x[1])))

    def reset(self):
        self._lst = []

    @property
    def time_stamps(self):
        return [x for x, _ in self._lst]

    @property
    def energy_values(self):
        return [x for _, x in self._lst]

    def __add__(self, other):
        res = EnergyHistory()
        res._lst = self._lst + other._lst
        return res

    def __iadd__(self, other):
        self._lst += other._lst
        return self

    def __len__(self):
        return len(self._lst)


def append_history(func):
    traced = func.__name__ == "check"

    @functools.wraps(func)
    def wrapper(self, energy):
        if self._history is not None:
            self._history.append((time.time(), energy.value))
        st = func(self, energy)
        if traced and _trace.TRACE is not None:
            _trace.emit(getattr(self, "_trace_tag", None), (self._itcount, float(energy.value)))
        return st
    return wrapper


class GradientNormController(IterationController):
    def __init__(self, tol_abs_gradnorm=None, tol_rel_gradnorm=None, convergence_level=1,
                 iteration_limit=None, name=None):
        super().__init__()
        self._tol_abs_gradnorm = tol_abs_gradnorm
        self._tol_rel_gradnorm = tol_rel_gradnorm
        self._convergence_level = convergence_level
        self._iteration_limit = iteration_limit
        self._name = name

    @property
    def needs_gradient_norm(self):
        return self._tol_abs_gradnorm is not None or self._tol_rel_gradnorm is not None

    @append_history
    def start(self, energy):
        self._itcount = -1
        self._ccount = 0
        if self._tol_rel_gradnorm is not None:
            self._tol_rel_gradnorm_now = self._tol_rel_gradnorm * energy.gradient_norm
        return self.check(energy)

    @append_history
    def check(self, energy):
        self._itcount += 1
        inclvl = False
        if self._tol_abs_gradnorm is not None:
            if energy.gradient_norm <= self._tol_abs_gradnorm:
                inclvl = True
        if self._tol_rel_gradnorm is not None:
            if energy.gradient_norm <= self._tol_rel_gradnorm_now:
                inclvl = True
        if inclvl:
            self._ccount += 1
        else:
            self._ccount = max(0, self._ccount - 1)
        if self._name is not None:
            logger.info("{}: Iteration #{} energy={:.6E} gradnorm={:.2E} clvl={}".format(
                self._name, self._itcount, energy.value, energy.gradient_norm, self._ccount))
        if self._iteration_limit is not None:
            if self._itcount >= self._iteration_limit:
                logger.warning("{}Iteration limit reached. Assuming convergence".format(
                    "" if self._name is None else self._name + ": "))
                return self.CONVERGED
        if self._ccount >= self._convergence_level:
            return self.CONVERGED
        return self.CONTINUE


class GradInfNormController(IterationController):
    def __init__(self, tol, convergence_level=1, iteration_limit=None, name=None):
        super().__init__()
        self._tol = tol
        self._convergence_level = convergence_level
        self._iteration_limit = iteration_limit
        self._name = name

    @append_history
    def start(self, energy):
        self._itcount = -1
        self._ccount = 0
        return self.check(energy)

    @append_history
    def check(self, energy):
        self._itcount += 1
        crit = energy.gradient.norm(np.inf) / abs(energy.value)
        if self._tol is not None and crit <= self._tol:
            self._ccount += 1
        else:
            self._ccount = max(0, self._ccount - 1)
        if self._iteration_limit is not None and self._itcount >= self._iteration_limit:
            logger.warning("Iteration limit reached. Assuming convergence")
            return self.CONVERGED
        if self._ccount >= self._convergence_level:
            return self.CONVERGED
        return self.CONTINUE


class DeltaEnergyController(IterationController):
    def __init__(self, tol_rel_deltaE, convergence_level=1, iteration_limit=None, name=None):
        super().__init__()
        self._tol_rel_deltaE = tol_rel_deltaE
        self._convergence_level = convergence_level
        self._iteration_limit = iteration_limit
        self._name = name

    @append_history
    def start(self, energy):
        self._itcount = -1
        self._ccount = 0
        self._Eold = 0.
        return self.check(energy)

    @append_history
    def check(self, energy):
        self._itcount += 1
        inclvl = False
        Eval = energy.value
        rel = abs(self._Eold - Eval) / max(abs(self._Eold), abs(Eval))
        if self._itcount > 0:
            if rel < self._tol_rel_deltaE:
                inclvl = True
        self._Eold = Eval
        if inclvl:
            self._ccount += 1
        else:
            self._ccount = max(0, self._ccount - 1)
        if self._iteration_limit is not None and self._itcount >= self._iteration_limit:
            logger.warning("Iteration limit reached. Assuming convergence")
            return self.CONVERGED
        if self._ccount >= self._convergence_level:
            return self.CONVERGED
        return self.CONTINUE


class AbsDeltaEnergyController(IterationController):
    def __init__(self, deltaE, convergence_level=1, iteration_limit=None, name=None):
        super().__init__()
        self._deltaE = deltaE
        self._convergence_level = convergence_level
        self._iteration_limit = iteration_limit
        self._name = name

    needs_gradient_norm = False

    @append_history
    def start(self, energy):
        self._itcount = -1
        self._ccount = 0
        self._Eold = 0.
        return self.check(energy)

    @append_history
    def check(self, energy):
        self._itcount += 1
        inclvl = False
        Eval = energy.value
        diff = abs(self._Eold - Eval)
        if self._itcount > 0:
            if diff < self._deltaE:
                inclvl = True
        self._Eold = Eval
        if inclvl:
            self._ccount += 1
        else:
            self._ccount = max(0, self._ccount - 1)
        if self._name is not None:
            logger.info("{}: Iteration #{} energy={:.6E} diff={:.6E} crit={:.1E} clvl={}".format(
                self._name, self._itcount, Eval, diff, self._deltaE, self._ccount))
        if self._iteration_limit is not None:
            if self._itcount >= self._iteration_limit:
                logger.warning("{} Iteration limit reached. Assuming convergence".format(
                    "" if self._name is None else self._name + ": "))
                return self.CONVERGED
        if self._ccount >= self._convergence_level:
            return self.CONVERGED
        return self.CONTINUE
