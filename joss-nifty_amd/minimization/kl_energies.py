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
from ..field import Field
from ..multi_domain import MultiDomain
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
    if napprox >= 1:
        # diagonal preconditioner from napprox metric samples
        # (kl_energies.py:127-128, probing.py:142-152); the draws use the
        # current RNG state before the sample seeds are spawned
        from ..probing import approximation2endo
        from ..sugar import makeOp
        met._approximation = makeOp(approximation2endo(met, napprox))

    parent = random._sseq[-1]
    sseq = random.spawn_sseq(n_samples)
    if mirror_samples:
        sseq = reduce(lambda a, b: a + b, [[ss] * 2 for ss in sseq]) if n_samples > 0 else []
    local_samples, local_neg = [], []
    utilities.check_MPI_synced_random_state(comm)
    utilities.check_MPI_equality(sseq, comm)
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
    # a rank holding one sample refines it as a batch of one: per sample the
    # batched refinement's arithmetic does not depend on the batch, so a
    # sharded run draws the 1-rank run's samples bit for bit
    if geometric and hi - lo >= 1 and isinstance(sam_position, MultiField):
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
                en.sample = i - lo      # tags the decision trace (trace.py) only
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


def _reduce_field(field, keys):
    """kl_energies.py:41-44"""
    if isinstance(field, MultiField) and len(keys) > 0:
        return field.extract_by_keys(set(field.keys()) - set(keys))
    return field


def _reduce_by_keys(field, operator, keys):
    """Partially insert the constant keys of ``field`` into ``operator``
    (kl_energies.py:47-75): returns the variable part and the contracted
    operator."""
    if isinstance(field, MultiField):
        cst_field = field.extract_by_keys(keys)
        var_field = field.extract_by_keys(set(field.keys()) - set(keys))
        _, operator = operator.simplify_for_constant_input(cst_field)
        return var_field, operator
    myassert(len(keys) == 0)
    return field, operator


def SampledKLEnergy(position, hamiltonian, n_samples, minimizer_sampling, mirror_samples=True,
                    constants=[], point_estimates=[], napprox=0, comm=None, nanisinf=True):
    """kl_energies.py:161-292.  ``constants`` are kept fixed during the KL
    minimisation, ``point_estimates`` are not sampled; a key in both is
    inserted into the Hamiltonian and removed from the KL (``invariants``)."""
    from .descent_minimizers import DescentMinimizer
    if not isinstance(hamiltonian, StandardHamiltonian):
        raise TypeError
    if hamiltonian.domain is not position.domain:
        raise ValueError
    if not isinstance(n_samples, int):
        raise TypeError
    if not isinstance(mirror_samples, bool):
        raise TypeError
    if not (minimizer_sampling is None or isinstance(minimizer_sampling, DescentMinimizer)):
        raise TypeError
    if isinstance(position, MultiField):
        if not set(constants).issubset(set(position.keys())):
            raise ValueError("Constants are not a subset of the keys of the latent space\n"
                             f"Latent space keys: {position.keys()}\nConstants keys: {constants}")
        if not set(point_estimates).issubset(set(position.keys())):
            raise ValueError("Point estimates are not a subset of the keys of the latent space\n"
                             f"Latent space keys: {position.keys()}\n"
                             f"Point estimate keys: {point_estimates}")
        if set(point_estimates) == set(position.keys()):
            raise RuntimeError("Point estimates for whole domain. Use EnergyAdapter instead.")
    invariant = list(set(constants).intersection(point_estimates))
    if isinstance(position, MultiField) and len(invariant) > 0:
        inv_pos = position.extract_by_keys(invariant)
    else:
        inv_pos = None
    position, hamiltonian = _reduce_by_keys(position, hamiltonian, invariant)
    _, ham_sampling = _reduce_by_keys(position, hamiltonian, point_estimates)
    sample_list = draw_samples(position, ham_sampling, minimizer_sampling, n_samples, mirror_samples,
                               napprox=napprox, comm=comm)
    return SampledKLEnergyClass(sample_list, hamiltonian, constants, inv_pos, nanisinf)


class SampledKLEnergyClass(Energy):
    """KL value/gradient averaged over samples (kl_energies.py:295-356)."""

    def __init__(self, sample_list, hamiltonian, constants, invariants, nanisinf):
        myassert(isinstance(sample_list, ResidualSampleList))
        myassert(sample_list.domain is hamiltonian.domain)
        if isinstance(sample_list._m, MultiField):
            if not (invariants is None or isinstance(invariants, MultiField)):
                raise TypeError
        super().__init__(_reduce_field(sample_list._m, constants))
        self._sample_list = sample_list
        self._hamiltonian = hamiltonian
        self._nanisinf = bool(nanisinf)
        self._constants = constants
        self._invariants = invariants

        def _func(inp):
            inp, tmp = _reduce_by_keys(inp, hamiltonian, constants)
            tmp = tmp(Linearization.make_var(inp))
            return tmp.val.val.real.item(), tmp.gradient
        # all local samples' H value / gradient in one batched pass where the
        # likelihood allows (geovi_batch.kl_batch), else per sample
        from . import geovi_batch
        kb = None
        if isinstance(sample_list._m, MultiField) and len(constants) == 0:
            kb = geovi_batch.kl_batch(hamiltonian, list(sample_list.local_iterator()))
        dom = self.position.domain

        def template():
            # a rank without samples joins the one all-reduce with zeros
            from ..multi_field import MultiField
            return 0.0, (MultiField.full(dom, 0.) if isinstance(dom, MultiDomain) else Field.full(dom, 0.))
        if kb is not None:
            self._val, self._grad = sample_list._average_results(list(zip(*kb)), template)
        else:
            self._val, self._grad = sample_list._average_tuple(_func, template)
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
        """Sample average of the Hamiltonian metric (kl_energies.py:340-350).
        Covered likelihoods: the local samples' metrics are linearised once per
        KL position and applied batched (geovi_batch.kl_metric_batch), the
        per-sample results summed in the reference's pairwise order and
        reduced across ranks with ONE all-reduce per application; otherwise
        the reference's per-sample Linearization path."""
        sl = self._sample_list
        if not hasattr(self, "_mbatch"):
            self._mbatch = None
            if isinstance(sl._m, MultiField) and len(self._constants) == 0 and sl.n_local_samples > 0:
                from . import geovi_batch
                self._mbatch = geovi_batch.kl_metric_batch(self._hamiltonian, list(sl.local_iterator()))
        if self._mbatch is not None:
            res = self._mbatch(x)
            return utilities.allreduce_sum(res, sl.comm, counts=sl._counts,
                                           template=lambda: 0 * x) / sl.n_samples

        def _func(inp):
            inp, tmp = _reduce_by_keys(inp, self._hamiltonian, self._constants)
            tmp = tmp(Linearization.make_var(inp, want_metric=True))
            return tmp.metric(x)
        return self._sample_list.average(_func)

    @property
    def metric(self):
        from ..operators.kl_metric import KLMetric
        return KLMetric(self)

    @property
    def samples(self):
        if self._invariants is None:
            return self._sample_list
        return self._sample_list.at(self._invariants)
