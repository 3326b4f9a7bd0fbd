"""MGVI/geoVI sample drawing and the sampled KL energy
(src/minimization/kl_energies.py:90-356).

``draw_samples`` follows the reference step by step: seed spawning and
mirroring (:131-133), shareRange sharding over ranks (:140-141, one process per
GPU), per-sample RNG contexts, SamplingEnabler.special_draw_sample (linear
MGVI residual; its CG runs fused on the device when the metric allows,
minimization/fused_cg.py) and, for geoVI, the NewtonCG refinement of
GaussianEnergy(m) @ transformation (:147-155)."""
from functools import reduce

import numpy as np

from .. import random, utilities
from ..linearization import Linearization
from ..multi_field import MultiField
from ..operators.energy_operators import GaussianEnergy, StandardHamiltonian
from ..operators.sampling_enabler import SamplingEnabler
from ..operators.sandwich_operator import SandwichOperator
from ..operators.scaling_operator import ScalingOperator
from ..utilities import get_MPI_params_from_comm, myassert, shareRange
from .energy import Energy
from .energy_adapter import EnergyAdapter
from .sample_list import ResidualSampleList


def draw_samples(position, H, minimizer, n_samples, mirror_samples, napprox=0, want_error=False, comm=None):
    if not isinstance(n_samples, int):
        raise TypeError
    if not isinstance(mirror_samples, bool):
        raise TypeError
    if not isinstance(H, StandardHamiltonian):
        raise TypeError
    if napprox != 0:
        raise NotImplementedError("napprox preconditioning is a 'next' item (SURVEY.md §8(f))")
    sam_position = position.extract(H.domain) if isinstance(position, MultiField) else position

    geometric = minimizer is not None
    if geometric:
        tr = H.likelihood_energy.get_transformation()
        if tr is None:
            raise ValueError("Geometric sampling only works for likelihoods")
        dtype, f_lh = tr
        scale = ScalingOperator(f_lh.target, 1., dtype)
        fl = f_lh(Linearization.make_var(sam_position))
        transformation = ScalingOperator(f_lh.domain, 1.) + fl.jac.adjoint @ f_lh
        transformation_mean = sam_position + fl.jac.adjoint(fl.val)
        met = SamplingEnabler(SandwichOperator.make(fl.jac, scale),
                              ScalingOperator(fl.domain, 1., float), H.iteration_controller)
    else:
        met = H(Linearization.make_var(sam_position, want_metric=True)).metric

    parent = random._sseq[-1]
    sseq = random.spawn_sseq(n_samples)
    if mirror_samples:
        sseq = reduce(lambda a, b: a + b, [[ss] * 2 for ss in sseq]) if n_samples > 0 else []
    local_samples, local_neg = [], []
    utilities.check_MPI_synced_random_state(comm)
    y = None
    ntask, rank, _ = get_MPI_params_from_comm(comm)
    lo, hi = shareRange(len(sseq), ntask, rank)
    # The local samples' linear solves are independent and share the metric:
    # draw every right-hand side first (each in its own RNG context, as the
    # reference does), solve them together (FusedCGBatch: one batched matvec
    # per CG iteration for all of them), then refine / collect each sample in
    # order.  Per sample the arithmetic is that of the reference's loop.
    drawing = [i for i in range(lo, hi) if not (mirror_samples and i % 2 != 0) or i == lo]
    batched = hasattr(met, "draw_rhs")
    prepared, prefetched = {}, False
    for i in drawing:
        ctx = random.Context(sseq[i])
        with ctx:
            prepared[i] = met.draw_rhs(True) if batched else met.special_draw_sample(True)
        if not prefetched:
            # host RNG off the critical path: replay this sample's draws for
            # the remaining local seeds and the next call's seeds
            prefetched = True
            nxt = random.predict_spawn(n_samples, parent)
            if mirror_samples:
                nxt = [ss for ss in nxt for _ in range(2)]
            todo = _distinct([sseq[j] for j in drawing if sseq[j] is not sseq[i]]) + _distinct(nxt[lo:hi])
            random.prefetch(todo, ctx.script)
    if batched:
        sols = met.solve_rhs([prepared[i] for i in drawing])
        prepared = dict(zip(drawing, sols))
    y = None
    gb = None
    if geometric and hi - lo > 1 and isinstance(sam_position, MultiField):
        from . import geovi_batch
        gb = geovi_batch.plan(minimizer, f_lh, None, sam_position)
    if gb is not None:
        # all local samples' NewtonCG refinements in lock step (geovi_batch):
        # per sample the reference's minimizer logic, requests batched
        lay = gb.layout
        starts, means = [], []
        for i in range(lo, hi):
            neg = mirror_samples and (i % 2 != 0)
            if not neg or y is None:
                y, yi = prepared[i]
                yp, yip = lay.pack(y), lay.pack(yi)
            means.append(gb.tmean - yp if neg else gb.tmean + yp)
            starts.append(gb.x0[0] - yip if neg else gb.x0[0] + yip)
        for xf in gb.refine(starts, means):
            local_samples.append(lay.unpack(xf - gb.x0[0]))
            local_neg.append(False)
        return ResidualSampleList(position, local_samples, local_neg, comm)
    for i in range(lo, hi):
        with random.Context(sseq[i]):
            neg = mirror_samples and (i % 2 != 0)
            if not neg or y is None:
                y, yi = prepared[i]
            if geometric:
                m = transformation_mean - y if neg else transformation_mean + y
                pos = sam_position - yi if neg else sam_position + yi
                en = GaussianEnergy(m) @ transformation
                en = EnergyAdapter(pos, en, nanisinf=True, want_metric=True)
                en, _ = minimizer(en)
                local_samples.append(en.position - sam_position)
                local_neg.append(False)
            else:
                local_samples.append(yi)
                local_neg.append(neg)
    return ResidualSampleList(position, local_samples, local_neg, comm)


def _distinct(seqs):
    out, seen = [], set()
    for ss in seqs:
        if id(ss) not in seen:
            seen.add(id(ss))
            out.append(ss)
    return out


def SampledKLEnergy(position, hamiltonian, n_samples, minimizer_sampling, mirror_samples=True,
                    constants=[], point_estimates=[], napprox=0, comm=None, nanisinf=True):
    if not isinstance(hamiltonian, StandardHamiltonian):
        raise TypeError
    if hamiltonian.domain is not position.domain:
        raise ValueError
    if len(constants) or len(point_estimates):
        raise NotImplementedError("constants/point_estimates are a 'next' item (SURVEY.md §8(f))")
    sample_list = draw_samples(position, hamiltonian, minimizer_sampling, n_samples, mirror_samples,
                               napprox=napprox, comm=comm)
    return SampledKLEnergyClass(sample_list, hamiltonian, constants, None, nanisinf)


class SampledKLEnergyClass(Energy):
    """KL value/gradient averaged over samples (kl_energies.py:295-356)."""

    def __init__(self, sample_list, hamiltonian, constants, invariants, nanisinf):
        myassert(isinstance(sample_list, ResidualSampleList))
        super().__init__(sample_list._m)
        self._sample_list = sample_list
        self._hamiltonian = hamiltonian
        self._nanisinf = bool(nanisinf)
        self._constants = constants
        self._invariants = invariants

        def _func(inp):
            tmp = hamiltonian(Linearization.make_var(inp))
            return tmp.val.val.real.item(), tmp.gradient
        # all local samples' H value / gradient in one batched pass where the
        # likelihood allows (geovi_batch.kl_batch), else per sample
        from . import geovi_batch
        pos = list(sample_list.local_iterator())
        kb = geovi_batch.kl_batch(hamiltonian, pos) if isinstance(sample_list._m, MultiField) else None
        if kb is not None:
            self._val, self._grad = sample_list._average_results(list(zip(*kb)))
        else:
            self._val, self._grad = sample_list._average_tuple(_func)
        if np.isnan(self._val) and self._nanisinf:
            self._val = np.inf

    @property
    def value(self):
        return self._val

    @property
    def gradient(self):
        return self._grad

    def at(self, position):
        return SampledKLEnergyClass(self._sample_list.at(position), self._hamiltonian, self._constants,
                                    self._invariants, self._nanisinf)

    def apply_metric(self, x):
        def _func(inp):
            tmp = self._hamiltonian(Linearization.make_var(inp, want_metric=True))
            return tmp.metric(x)
        return self._sample_list.average(_func)

    @property
    def metric(self):
        from ..operators.kl_metric import KLMetric
        return KLMetric(self)

    @property
    def samples(self):
        return self._sample_list
