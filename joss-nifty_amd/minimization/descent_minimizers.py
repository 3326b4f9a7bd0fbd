"""DescentMinimizer / NewtonCG (src/minimization/descent_minimizers.py:24-206);
the geoVI nonlinear sample refinement runs NewtonCG on
GaussianEnergy(m) @ transformation (kl_energies.py:147-155)."""
from ..logger import logger
from . import trace
from .conjugate_gradient import ConjugateGradient
from .iteration_controllers import AbsDeltaEnergyController, GradientNormController
from .line_search import LineSearch
from .minimizer import Minimizer
from .quadratic_energy import QuadraticEnergy


class DescentMinimizer(Minimizer):
    def __init__(self, controller, line_searcher=LineSearch()):
        self._controller = controller
        self.line_searcher = line_searcher

    def __call__(self, energy):
        gen = self.minimize_gen(energy)
        try:
            req = next(gen)
            while True:
                req = gen.send(self.serve(req))
        except StopIteration as e:
            return e.value

    def serve(self, req):
        """Synchronous evaluation of one request of minimize_gen."""
        if req[0] == "dir":
            self._trace_sample = req[3]
            return self.get_descent_direction(req[1], req[2])
        return self.line_searcher.serve(req)

    def minimize_gen(self, energy):
        """DescentMinimizer.__call__ (descent_minimizers.py:52-108) as a
        generator of requests: ("dir", energy, f_k_minus_1, sample) -> descent
        direction, plus the line search's ("dd", ...) / ("at", ...).
        ``sample`` (energy.sample of the starting energy, if set) only tags
        the decision trace (minimization/trace.py)."""
        f_k_minus_1 = None
        controller = self._controller
        stag = getattr(energy, "sample", None)
        trace.tag(controller, ("newton", stag))
        status = controller.start(energy)
        if status != controller.CONTINUE:
            return energy, status
        while True:
            if energy.gradient_norm == 0:
                return energy, controller.CONVERGED
            pk = yield ("dir", energy, f_k_minus_1, stag)
            ls = self.line_searcher.perform_line_search_gen(energy=energy, pk=pk, f_k_minus_1=f_k_minus_1)
            if trace.active():
                ls = _traced_trials(ls, stag)
            new_energy, success = yield from ls
            if not success:
                self.reset()
            f_k_minus_1 = energy.value
            if new_energy.value > energy.value:
                logger.error("Error: Energy has increased")
                return energy, controller.ERROR
            if new_energy.value == energy.value:
                logger.warning("Warning: Energy has not changed. Assuming convergence...")
                return new_energy, controller.CONVERGED
            energy = new_energy
            status = self._controller.check(energy)
            if status != controller.CONTINUE:
                return energy, status

    def reset(self):
        pass

    def get_descent_direction(self, energy, old_value=None):
        raise NotImplementedError


def _traced_trials(gen, stag):
    """pass a line-search generator through, recording its trial steps and
    the energies found there"""
    trace.emit(("trial", stag), None)
    trace.emit(("trialE", stag), None)
    try:
        req = next(gen)
        while True:
            if req[0] == "at":
                trace.emit(("trial", stag), float(req[2]))
            try:
                ans = yield req
            except Exception as exc:     # noqa: BLE001 -- forwarded to the search
                req = gen.throw(exc)
                continue
            if req[0] == "at":
                trace.emit(("trialE", stag), float(ans.value))
            elif req[0] == "dd":
                trace.emit(("trialD", stag), (float(req[1].value), float(ans)))
            req = gen.send(ans)
    except StopIteration as e:
        return e.value


class SteepestDescent(DescentMinimizer):
    def get_descent_direction(self, energy, _=None):
        return -energy.gradient


class NewtonCG(DescentMinimizer):
    def __init__(self, controller, napprox=0, line_searcher=None, name=None, nreset=20,
                 max_cg_iterations=200, energy_reduction_factor=0.1, enable_logging=False):
        if line_searcher is None:
            line_searcher = LineSearch(preferred_initial_step_size=1.)
        super().__init__(controller=controller, line_searcher=line_searcher)
        self._napprox = napprox
        self._name = name
        self._nreset = nreset
        self._max_cg_iterations = max_cg_iterations
        self._alpha = energy_reduction_factor
        from .iteration_controllers import EnergyHistory
        self._history = EnergyHistory() if enable_logging else None

    def get_descent_direction(self, energy, old_value=None):
        if old_value is None:
            ic = GradientNormController(iteration_limit=5)
        else:
            ediff = self._alpha * (old_value - energy.value)
            ic = AbsDeltaEnergyController(ediff, iteration_limit=self._max_cg_iterations, name=self._name)
        trace.tag(ic, ("dir", getattr(self, "_trace_sample", None)))
        if self._history is not None:
            ic.enable_logging()
        # CG from x0 = 0: the metric is linear, so A(x0) - b is -b and the
        # reference's metric application on the zero vector is skipped
        g = energy.gradient
        e = QuadraticEnergy(0 * energy.position, energy.metric, g, _grad=-g)
        e, conv = ConjugateGradient(ic, nreset=self._nreset)(e, None)
        if self._history is not None:
            self._history += ic.history
        if conv == ic.ERROR:
            raise ValueError("Cannot find descent direction")
        return -e.position

    @property
    def inversion_history(self):
        return self._history
