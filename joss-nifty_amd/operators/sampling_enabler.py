"""SamplingEnabler (src/operators/sampling_enabler.py:24-89): draws from the
inverse of likelihood + prior metric by CG from a prior sample."""
from ..minimization import trace
from ..minimization.conjugate_gradient import ConjugateGradient
from ..minimization.quadratic_energy import QuadraticEnergy
from .endomorphic_operator import EndomorphicOperator
from .operator import Operator


class SamplingEnabler(EndomorphicOperator):
    def __init__(self, likelihood, prior, iteration_controller, approximation=None, start_from_zero=False):
        if not isinstance(likelihood, Operator) or not isinstance(prior, Operator):
            raise TypeError
        self._likelihood = likelihood
        self._prior = prior
        self._ic = iteration_controller
        self._approximation = approximation
        self._start_from_zero = bool(start_from_zero)
        self._op = likelihood + prior
        self._domain = self._op.domain
        self._capability = self._op.capability
        self.apply = self._op.apply

    def draw_rhs(self, from_inverse=True):
        """First half of special_draw_sample: the random draws and the CG
        problem.  Returns ("done", (b, x)) when the operator samples directly,
        else ("cg", energy)."""
        try:
            res = self._op.draw_sample(from_inverse)
            return "done", (self._op(res), res)
        except NotImplementedError:
            if not from_inverse:
                raise ValueError("from_inverse must be True here")
            if self._start_from_zero:
                b = self._op.draw_sample()
                return "cg", QuadraticEnergy(0 * b, self._op, b)
            s = self._prior.draw_sample(from_inverse=True)
            nj = self._likelihood.draw_sample()
            b = self._prior(s) + nj
            return "cg", QuadraticEnergy(s, self._op, b, _grad=self._likelihood(s) - nj)

    def solve_rhs(self, prepared):
        """Second half for a list of draw_rhs results: the CG solves, batched
        into one lock-step solve (minimization/fused_cg.FusedCGBatch) when the
        metric allows, otherwise one after another.  Returns [(b, x)]."""
        import copy
        out = [None] * len(prepared)
        todo = [j for j, (kind, _) in enumerate(prepared) if kind == "cg"]
        for j, (kind, v) in enumerate(prepared):
            if kind == "done":
                out[j] = v
        if not todo:
            return out
        energies = [prepared[j][1] for j in todo]
        res = None
        if self._approximation is None and len(todo) > 1:
            from ..minimization.fused_cg import fused_cg_batch_or_none
            ctls = [trace.tag(copy.deepcopy(self._ic), ("lin", j)) for j in todo]
            res = fused_cg_batch_or_none(energies, ctls, ConjugateGradient(self._ic)._nreset)
        if res is None:
            res = []
            for j, e in zip(todo, energies):
                trace.tag(self._ic, ("lin", j))
                inverter = ConjugateGradient(self._ic)
                if self._approximation is not None:
                    res.append(inverter(e, preconditioner=self._approximation.inverse))
                else:
                    res.append(inverter(e))
        for j, e, (en, _) in zip(todo, energies, res):
            out[j] = (e._b, en.position)
        return out

    def special_draw_sample(self, from_inverse=False):
        try:
            res = self._op.draw_sample(from_inverse)
            return self._op(res), res
        except NotImplementedError:
            if not from_inverse:
                raise ValueError("from_inverse must be True here")
            if self._start_from_zero:
                b = self._op.draw_sample()
                energy = QuadraticEnergy(0 * b, self._op, b)
            else:
                s = self._prior.draw_sample(from_inverse=True)
                nj = self._likelihood.draw_sample()
                b = self._prior(s) + nj
                energy = QuadraticEnergy(s, self._op, b, _grad=self._likelihood(s) - nj)
            inverter = ConjugateGradient(self._ic)
            if self._approximation is not None:
                energy, convergence = inverter(energy, preconditioner=self._approximation.inverse)
            else:
                energy, convergence = inverter(energy)
            return b, energy.position

    def draw_sample(self, from_inverse=False):
        return self.special_draw_sample(from_inverse=from_inverse)[1]
