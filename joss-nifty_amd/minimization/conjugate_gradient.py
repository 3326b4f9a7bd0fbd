"""Linear conjugate gradient (src/minimization/conjugate_gradient.py:24-126).

``ConjugateGradient.__call__`` keeps the reference's algorithm, guards and
controller protocol.  When the energy is a QuadraticEnergy whose metric is a
fusable sampling metric (shift * 1 + J^T W J with a fused model Jacobian J,
see operators/sandwich_operator.py) and no preconditioner is given, the
iteration runs on packed device vectors with the native CG kernels
(minimization/fused_cg.py): same recurrences, same nreset residual refresh,
same guard and controller decisions, one host sync per iteration."""
import numpy as np

from ..logger import logger
from .minimizer import Minimizer


class ConjugateGradient(Minimizer):
    iterations_total = 0  # CG iterations run by all instances (benchmark bookkeeping)

    def __init__(self, controller, nreset=20, allow_fused=True):
        self._controller = controller
        self._nreset = nreset
        self._allow_fused = allow_fused

    def __call__(self, energy, preconditioner=None):
        if self._allow_fused and preconditioner is None:
            from .fused_cg import fused_cg_or_none
            res = fused_cg_or_none(energy, self._controller, self._nreset)
            if res is not None:
                return res
        return self._generic(energy, preconditioner)

    def _generic(self, energy, preconditioner=None):
        controller = self._controller
        status = controller.start(energy)
        if status != controller.CONTINUE:
            return energy, status

        r = energy.gradient
        d = r if preconditioner is None else preconditioner(r)

        previous_gamma = r.s_vdot(d).real
        if np.isnan(previous_gamma):
            logger.error("Error: ConjugateGradient: previous_gamma==NaN")
            return energy, controller.ERROR
        if previous_gamma == 0:
            return energy, controller.CONVERGED

        ii = 0
        while True:
            q = energy.apply_metric(d)
            curv = d.s_vdot(q).real
            if np.isnan(curv):
                logger.error("Error: ConjugateGradient: curv==NaN")
                return energy, controller.ERROR
            if curv == 0.:
                logger.error("Error: ConjugateGradient: curv==0.")
                return energy, controller.ERROR
            alpha = previous_gamma / curv
            if alpha < 0:
                logger.error("Error: ConjugateGradient: alpha<0.")
                return energy, controller.ERROR

            ii += 1
            ConjugateGradient.iterations_total += 1
            if ii < self._nreset:
                r = r - q * alpha
                energy = energy.at_with_grad(energy.position - alpha * d, r)
            else:
                energy = energy.at(energy.position - alpha * d)
                r = energy.gradient
                ii = 0

            s = r if preconditioner is None else preconditioner(r)
            gamma = r.s_vdot(s).real
            if np.isnan(gamma):
                logger.error("Error: ConjugateGradient: gamma==NaN")
                return energy, controller.ERROR
            if gamma < 0:
                logger.error("Positive definiteness of preconditioner violated!")
                return energy, controller.ERROR
            if gamma == 0:
                return energy, controller.CONVERGED

            status = controller.check(energy)
            if status != controller.CONTINUE:
                return energy, status

            d = d * max(0, gamma / previous_gamma) + s
            previous_gamma = gamma
