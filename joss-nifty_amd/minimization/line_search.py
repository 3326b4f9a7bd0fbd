"""Strong-Wolfe line search (src/minimization/line_search.py:24-420), written as a
generator of evaluation requests (see LineSearch.perform_line_search_gen)."""
import numpy as np

from ..logger import logger


class LineEnergy:
    def __init__(self, line_position, energy, line_direction, offset=0.):
        self._line_position = float(line_position)
        self._line_direction = line_direction
        if self._line_position == float(offset):
            self._energy = energy
        else:
            pos = energy.position + (self._line_position - float(offset)) * self._line_direction
            self._energy = energy.at(position=pos)

    def at(self, line_position):
        return LineEnergy(line_position, self._energy, self._line_direction, offset=self._line_position)

    @property
    def energy(self):
        return self._energy

    @property
    def value(self):
        return self._energy.value

    @property
    def directional_derivative(self):
        res = self._energy.gradient.s_vdot(self._line_direction)
        if abs(np.imag(res)) / max(abs(res), 1.) > 1e-12:
            logger.warning(f"directional derivative has non-negligible imaginary part: {res}")
        return float(np.real(res))


class LineSearch:
    def __init__(self, preferred_initial_step_size=None, c1=1e-4, c2=0.9, max_step_size=1e30,
                 max_iterations=100, max_zoom_iterations=100):
        self.preferred_initial_step_size = preferred_initial_step_size
        self.c1 = float(c1)
        self.c2 = float(c2)
        self.max_step_size = max_step_size
        self.max_iterations = int(max_iterations)
        self.max_zoom_iterations = int(max_zoom_iterations)

    # The search is written as a generator of evaluation requests so that the
    # geoVI refinement of several samples can serve them in batches
    # (minimization/geovi_batch.py) with exactly this per-sample logic:
    #   ("dd", energy, pk)        -> directional derivative  energy.gradient . pk
    #   ("at", energy0, alpha, pk) -> the energy at energy0.position + alpha * pk
    # (LineEnergy, line_search.py:24-80: le_0.at(alpha) with offset 0).
    # perform_line_search drives it with immediate evaluations.

    @staticmethod
    def serve(req):
        """Synchronous evaluation of one request (LineEnergy semantics)."""
        if req[0] == "dd":
            return LineEnergy(0., req[1], req[2], 0.).directional_derivative
        if req[0] == "at":
            return LineEnergy(0., req[1], req[3], 0.).at(req[2]).energy
        raise ValueError(req[0])

    def perform_line_search(self, energy, pk, f_k_minus_1=None):
        gen = self.perform_line_search_gen(energy, pk, f_k_minus_1)
        try:
            req = next(gen)
            while True:
                req = gen.send(self.serve(req))
        except StopIteration as e:
            return e.value

    def perform_line_search_gen(self, energy, pk, f_k_minus_1=None):
        le_0 = energy
        maxstepsize = energy.longest_step(pk)
        if maxstepsize is None:
            maxstepsize = self.max_step_size
        maxstepsize = min(maxstepsize, self.max_step_size)
        old_phi_0 = f_k_minus_1
        phi_0 = le_0.value
        phiprime_0 = yield ("dd", le_0, pk)
        if phiprime_0 == 0:
            logger.warning("Directional derivative is zero; assuming convergence")
            return energy, False
        if phiprime_0 > 0:
            logger.error("Error: search direction is not a descent direction")
            return energy, False
        alpha0 = 0.
        phi_alpha0 = phi_0
        phiprime_alpha0 = phiprime_0
        if self.preferred_initial_step_size is not None:
            alpha1 = self.preferred_initial_step_size
        elif old_phi_0 is not None:
            alpha1 = min(1.0, 1.01 * 2 * (phi_0 - old_phi_0) / phiprime_0)
            if alpha1 < 0:
                alpha1 = 1.0
        else:
            alpha1 = 1.0 / pk.norm()
        alpha1 = min(alpha1, 0.99 * maxstepsize)
        iteration_number = 0
        le_alpha1 = None
        while iteration_number < self.max_iterations:
            iteration_number += 1
            if alpha1 == 0:
                return le_0, False
            try:
                le_alpha1 = yield ("at", le_0, alpha1, pk)
                phi_alpha1 = le_alpha1.value
            except FloatingPointError:
                alpha1 = (alpha0 + alpha1) / 2
                continue
            if np.isnan(phi_alpha1) or np.abs(phi_alpha1) > 1e100:
                alpha1 = (alpha0 + alpha1) / 2
                continue
            if (phi_alpha1 > phi_0 + self.c1 * alpha1 * phiprime_0) or \
                    ((phi_alpha1 >= phi_alpha0) and (iteration_number > 1)):
                return (yield from self._zoom(alpha0, alpha1, phi_0, phiprime_0, phi_alpha0, phiprime_alpha0,
                                              phi_alpha1, le_0, pk))
            phiprime_alpha1 = yield ("dd", le_alpha1, pk)
            if abs(phiprime_alpha1) <= -self.c2 * phiprime_0:
                return le_alpha1, True
            if phiprime_alpha1 >= 0:
                return (yield from self._zoom(alpha1, alpha0, phi_0, phiprime_0, phi_alpha1, phiprime_alpha1,
                                              phi_alpha0, le_0, pk))
            alpha0, alpha1 = alpha1, min(2 * alpha1, maxstepsize)
            if alpha1 == maxstepsize:
                logger.warning("max step size reached")
                return le_alpha1, False
            phi_alpha0 = phi_alpha1
            phiprime_alpha0 = phiprime_alpha1
        logger.warning("max iterations reached")
        return le_alpha1, False

    def _zoom(self, alpha_lo, alpha_hi, phi_0, phiprime_0, phi_lo, phiprime_lo, phi_hi, le_0, pk):
        cubic_delta = 0.2
        quad_delta = 0.1
        alpha_recent = None
        phi_recent = None
        if phi_lo > phi_0 + self.c1 * alpha_lo * phiprime_0:
            raise ValueError("inconsistent data")
        if phiprime_lo * (alpha_hi - alpha_lo) >= 0.:
            raise ValueError("inconsistent data")
        for i in range(self.max_zoom_iterations):
            delta_alpha = alpha_hi - alpha_lo
            a, b = min(alpha_lo, alpha_hi), max(alpha_lo, alpha_hi)
            if i > 0:
                cubic_check = cubic_delta * delta_alpha
                alpha_j = self._cubicmin(alpha_lo, phi_lo, phiprime_lo, alpha_hi, phi_hi, alpha_recent, phi_recent)
            if (i == 0) or (alpha_j is None) or (alpha_j > b - cubic_check) or (alpha_j < a + cubic_check):
                quad_check = quad_delta * delta_alpha
                alpha_j = self._quadmin(alpha_lo, phi_lo, phiprime_lo, alpha_hi, phi_hi)
                if (alpha_j is None) or (alpha_j > b - quad_check) or (alpha_j < a + quad_check):
                    alpha_j = alpha_lo + 0.5 * delta_alpha
            le_alphaj = yield ("at", le_0, alpha_j, pk)
            phi_alphaj = le_alphaj.value
            if (phi_alphaj > phi_0 + self.c1 * alpha_j * phiprime_0) or (phi_alphaj >= phi_lo):
                alpha_recent, phi_recent = alpha_hi, phi_hi
                alpha_hi, phi_hi = alpha_j, phi_alphaj
            else:
                phiprime_alphaj = yield ("dd", le_alphaj, pk)
                if abs(phiprime_alphaj) <= -self.c2 * phiprime_0:
                    return le_alphaj, True
                if phiprime_alphaj * delta_alpha >= 0:
                    alpha_recent, phi_recent = alpha_hi, phi_hi
                    alpha_hi, phi_hi = alpha_lo, phi_lo
                else:
                    alpha_recent, phi_recent = alpha_lo, phi_lo
                alpha_lo, phi_lo, phiprime_lo = alpha_j, phi_alphaj, phiprime_alphaj
        else:
            logger.warning("The line search algorithm (zoom) did not converge.")
            return le_alphaj, False

    def _cubicmin(self, a, fa, fpa, b, fb, c, fc):
        with np.errstate(divide="raise", over="raise", invalid="raise"):
            try:
                C = fpa
                db = b - a
                dc = c - a
                denom = db * db * dc * dc * (db - dc)
                d1 = np.empty((2, 2))
                d1[0, 0] = dc * dc
                d1[0, 1] = -(db * db)
                d1[1, 0] = -(dc * dc * dc)
                d1[1, 1] = db * db * db
                [A, B] = np.dot(d1, np.asarray([fb - fa - C * db, fc - fa - C * dc]).ravel())
                A /= denom
                B /= denom
                radical = B * B - 3 * A * C
                xmin = a + (-B + np.sqrt(radical)) / (3 * A)
            except ArithmeticError:
                return None
        if not np.isfinite(xmin):
            return None
        return xmin

    def _quadmin(self, a, fa, fpa, b, fb):
        with np.errstate(divide="raise", over="raise", invalid="raise"):
            try:
                db = b - a * 1.0
                B = (fb - fa - fpa * db) / (db * db)
                xmin = a - fpa / (2.0 * B)
            except ArithmeticError:
                return None
        if not np.isfinite(xmin):
            return None
        return xmin
