"""Correlated-field amplitude building blocks
(src/library/correlated_fields.py:43-212).

The linear helpers (_SlopeRemover, _TwoLogIntegrations, _SpecialSum) are
provided as LinearOperators for API parity, and the same math is exposed as
plain tensor functions (``twolog``, ``twolog_adjoint``, ``slope_remove``...)
used by the fused amplitude model of correlated_fields_simple.py.  All of it
works on B-sized power-spectrum arrays (B = number of |k| bins), i.e. a small
fraction of the grid."""
import numpy as np
import torch

from ..domain_tuple import DomainTuple
from ..domains import PowerSpace, UnstructuredDomain
from ..field import Field
from ..operators.endomorphic_operator import EndomorphicOperator
from ..operators.linear_operator import LinearOperator
from ..sugar import makeDomain
from ..utilities import myassert


def _log_k_lengths(pspace):
    """log(k_lengths) without zeromode (correlated_fields.py:50-52)"""
    return np.log(pspace.k_lengths[1:])


def _relative_log_k_lengths(power_space):
    """log-distance to the first bin; [0]=[1]=0 (:55-64)"""
    if isinstance(power_space, DomainTuple):
        power_space = power_space[0]
    logkl = _log_k_lengths(power_space)
    logkl = logkl - logkl[0]
    return np.insert(logkl, 0, 0)


def _log_vol(power_space):
    """(:67-71)"""
    if isinstance(power_space, DomainTuple):
        power_space = power_space[0]
    logk = _log_k_lengths(power_space)
    return logk[1:] - logk[:-1]


# --------------------------------------------------------------- tensor math
def twolog(x0, x1, lv):
    """_TwoLogIntegrations TIMES on (2, B-2) -> (B,) (:127-143)."""
    c = torch.cumsum(x1, 0)
    cprev = torch.cat([c.new_zeros(1), c[:-1]])
    t = (c + cprev) / 2 * lv + x0
    return torch.cat([c.new_zeros(2), torch.cumsum(t, 0)])


def _revcumsum(v):
    return torch.flip(torch.cumsum(torch.flip(v, (0,)), 0), (0,))


def twolog_adjoint(g, lv):
    """_TwoLogIntegrations ADJOINT_TIMES on (B,) -> ((B-2,), (B-2,)) (:144-155)."""
    y = _revcumsum(g[2:])
    z = y * (lv / 2.)
    w = z + torch.cat([z[1:], z.new_zeros(1)])
    return y, _revcumsum(w)


def slope_remove(x, sc):
    """_SlopeRemover TIMES (:105-110)"""
    return x - x[-1] * sc


def slope_remove_adjoint(x, sc):
    """_SlopeRemover ADJOINT (:111-113)"""
    res = x.clone()
    res[-1] = res[-1] - torch.sum(x * sc)
    return res


# --------------------------------------------------------------- operators
def _dev_tensor(a):
    from .. import config
    return torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float64, device=config.device())


class _SlopeRemover(EndomorphicOperator):
    def __init__(self, domain, space=0):
        self._domain = makeDomain(domain)
        myassert(isinstance(self._domain[space], PowerSpace))
        if len(self._domain) != 1:
            raise NotImplementedError("only single-space power domains are supported")
        logkl = _relative_log_k_lengths(self._domain[space])
        self._sc = _dev_tensor(logkl / float(logkl[-1]))
        self._capability = self.TIMES | self.ADJOINT_TIMES

    def apply(self, x, mode):
        self._check_input(x, mode)
        if mode == self.TIMES:
            return Field(self._domain, slope_remove(x.val, self._sc))
        return Field(self._domain, slope_remove_adjoint(x.val, self._sc))


class _TwoLogIntegrations(LinearOperator):
    def __init__(self, target, space=0):
        self._target = makeDomain(target)
        myassert(isinstance(self.target[space], PowerSpace))
        if len(self._target) != 1:
            raise NotImplementedError("only single-space power domains are supported")
        self._domain = makeDomain(UnstructuredDomain((2, self.target[space].shape[0] - 2)))
        self._lv = _dev_tensor(_log_vol(self._target[space]))
        self._capability = self.TIMES | self.ADJOINT_TIMES

    def apply(self, x, mode):
        self._check_input(x, mode)
        if mode == self.TIMES:
            v = x.val
            return Field(self._target, twolog(v[0], v[1], self._lv))
        r0, r1 = twolog_adjoint(x.val, self._lv)
        return Field(self._domain, torch.stack([r0, r1]))


class _SpecialSum(EndomorphicOperator):
    def __init__(self, domain, space=0):
        self._domain = makeDomain(domain)
        self._capability = self.TIMES | self.ADJOINT_TIMES

    def apply(self, x, mode):
        self._check_input(x, mode)
        return Field(self._domain, torch.sum(x.val).expand(self._domain.shape).clone())


def mode_multiplicity(pspace):
    """pd.adjoint(full(1)) with the zero mode set to 0 (_Normalization :171-175)."""
    m = np.bincount(pspace.pindex.ravel(), minlength=pspace.shape[0]).astype(np.float64)
    m[0] = 0.
    return m


# ------------------------------------------------------- CorrelatedFieldMaker
def _structured_spaces(domain):
    """(correlated_fields.py:74-77)"""
    if isinstance(domain[0], UnstructuredDomain):
        return np.arange(1, len(domain))
    return np.arange(len(domain))


def _total_fluctuation_realized(samples):
    """(correlated_fields.py:80-88)"""
    from ..operators.contraction_operator import ContractionOperator
    spaces = _structured_spaces(samples[0].domain)
    co = ContractionOperator(samples[0].domain, spaces)
    size = co.domain.size / co.target.size
    res = 0.
    for s in samples:
        res = res + (s - co.adjoint(co(s) / size)) ** 2
    res = res.mean(spaces) / len(samples)
    return np.sqrt(res if np.isscalar(res) else res.val_np())


def _rg_only(dom):
    from ..domains import RGSpace
    return all(isinstance(d, RGSpace) for d in dom)


class _Amplitude:
    """Fluctuation amplitude of one `add_fluctuations` call
    (correlated_fields.py:276-386): entry 0 is `totvol`, entries k > 0 are
    fluctuations * totvol * An_k with An the square root of the normalised
    spectrum (_Normalization, :158-201).  The value and Jacobian come from the
    fused B-sized amplitude model of correlated_fields_simple (the same one
    SimpleCorrelatedField uses, no zero mode) followed by the constant
    `Adder(vol0)`; the latent keys are the reference's
    (`<prefix>fluctuations`, `...loglogavgslope`, `...flexibility`,
    `...asperity`, `...spectrum`)."""

    def __new__(cls, target_subdomain, harmonic_partner, fluctuations, flexibility, asperity,
                loglogavgslope, prefix):
        from ..operators.adder import Adder
        from ..operators.normal_operators import LognormalTransform
        from ..sugar import makeField
        from .correlated_fields_simple import _AmplitudeModel, _AmplitudeOperator
        model = _AmplitudeModel(target_subdomain[-1], harmonic_partner, None, fluctuations, flexibility,
                                asperity, loglogavgslope, prefix)
        raw = _AmplitudeOperator(model)
        vol0 = np.zeros(raw.target.shape)
        vol0[0] = model.total_vol
        op = Adder(makeField(raw.target, vol0)) @ raw
        op.model = model
        op.params = (fluctuations, flexibility, asperity, loglogavgslope, prefix)
        op.harmonic_partner = harmonic_partner
        op.fluctuation_amplitude = LognormalTransform(*fluctuations, prefix + "fluctuations", 0)
        op._space = 0
        return op


def _AmplitudeMatern(pow_spc, scale, cutoff, loglogslope, totvol):
    """Matern-kernel amplitude (correlated_fields.py:232-274) composed from
    generic operators: A(k) = a (1 + k^2 / b^2)^(c/4), volume factors as the
    reference."""
    from ..operators.adder import Adder
    from ..operators.contraction_operator import ContractionOperator
    from ..operators.diagonal_operator import DiagonalOperator
    from ..operators.simple_linear_operators import VdotOperator
    from ..sugar import full, makeField
    expander = ContractionOperator(pow_spc, spaces=None).adjoint
    k_squared = makeField(pow_spc, pow_spc.k_lengths ** 2)
    scale = expander @ scale.log()
    cutoff = VdotOperator(k_squared).adjoint @ cutoff.power(-2.)
    spectral_idx = expander.scale(0.25) @ loglogslope
    ker = Adder(full(pow_spc, 1.)) @ cutoff
    ker = spectral_idx * ker.log() + scale
    op = ker.exp()
    vol0, vol1 = np.zeros(pow_spc.shape), np.zeros(pow_spc.shape)
    vol0[0] = totvol
    vol1[1:] = totvol ** 0.5
    op = Adder(makeField(pow_spc, vol0)) @ DiagonalOperator(makeField(pow_spc, vol1)) @ op
    op.fluctuation_amplitude = op.power(2).integrate().sqrt()
    op._space = 0
    return op


class CorrelatedFieldMaker:
    """Builder for (product-spectrum) correlated fields
    (src/library/correlated_fields.py:388-1115), same methods, argument
    meaning, latent keys and errors.

    `finalize` of ONE `add_fluctuations` component on an RGSpace, with the
    zero mode either disabled (offset_std None) or LogNormal, returns the
    fused SimpleCorrelatedField operator (native prologue/epilogue Hartley
    engine, carried-CG Jacobian): the reference's operator tree for that case
    is algebraically the same map (test_complicated_vs_simple,
    test/test_operators/test_correlated_fields.py:214-272).  Every other case
    (product spectra, Matern components, a unit or operator-valued zero mode,
    a field offset) is built as the reference's operator tree
    (:764-823) on the device operators: per-component fused amplitudes,
    PowerDistributor + ContractionOperator broadcasts, and the native
    Hartley transform per sub-space.  `total_N > 0` (stacked field models,
    _Distributor / dofdex) is outside the hot path and raises."""

    def __init__(self, prefix, total_N=0):
        if total_N != 0:
            raise NotImplementedError("total_N > 0 (stacked correlated fields) is out of scope; "
                                      "see DESIGN.md")
        self._azm = None
        self._offset_mean = None
        self._offset_std = None
        self._a = []
        self._target_subdomains = []
        self._prefix = prefix
        self._total_N = total_N

    def add_fluctuations(self, target_subdomain, fluctuations, flexibility, asperity, loglogavgslope,
                         prefix='', index=None, dofdex=None, harmonic_partner=None):
        """(correlated_fields.py:430-595)"""
        if harmonic_partner is None:
            harmonic_partner = target_subdomain.get_default_codomain()
        else:
            target_subdomain.check_codomain(harmonic_partner)
            harmonic_partner.check_codomain(target_subdomain)
        if dofdex is not None and len(dofdex) != self._total_N:
            raise ValueError("length of dofdex needs to match total_N")
        target_subdomain = makeDomain(target_subdomain)
        for arg in (fluctuations, loglogavgslope):
            if len(arg) != 2:
                raise TypeError
        for kw, arg in (("flexibility", flexibility), ("asperity", asperity)):
            if arg is None:
                continue
            if len(arg) != 2:
                raise TypeError
            if arg[0] <= 0. or arg[1] <= 0.:
                raise ValueError(f"{kw} must be strictly positive (or None)")
        if flexibility is None and asperity is not None:
            raise ValueError("flexibility may not be disabled on its own")
        pre = self._prefix + str(prefix)
        amp = _Amplitude(target_subdomain, harmonic_partner, fluctuations, flexibility, asperity,
                         loglogavgslope, pre)
        if index is not None:
            self._a.insert(index, amp)
            self._target_subdomains.insert(index, target_subdomain)
        else:
            self._a.append(amp)
            self._target_subdomains.append(target_subdomain)

    def add_fluctuations_matern(self, target_subdomain, scale, cutoff, loglogslope, prefix='',
                                adjust_for_volume=True, harmonic_partner=None):
        """(correlated_fields.py:597-690)"""
        from ..operators.normal_operators import LognormalTransform, NormalTransform
        if harmonic_partner is None:
            harmonic_partner = target_subdomain.get_default_codomain()
        else:
            target_subdomain.check_codomain(harmonic_partner)
            harmonic_partner.check_codomain(target_subdomain)
        target_subdomain = makeDomain(target_subdomain)
        pre = self._prefix + prefix
        scale = LognormalTransform(*scale, pre + 'scale', 0)
        cutoff = LognormalTransform(*cutoff, pre + 'cutoff', 0)
        loglogslope = NormalTransform(*loglogslope, pre + 'loglogslope', 0)
        totvol = target_subdomain[-1].total_volume if adjust_for_volume else 1.
        amp = _AmplitudeMatern(PowerSpace(harmonic_partner), scale, cutoff, loglogslope, totvol)
        self._a.append(amp)
        self._target_subdomains.append(target_subdomain)

    def set_amplitude_total_offset(self, offset_mean, offset_std, dofdex=None):
        """(correlated_fields.py:692-762)"""
        from ..logger import logger
        from ..operators.normal_operators import LognormalTransform
        from ..operators.operator import Operator
        if self._offset_mean is not None and self._azm is not None:
            logger.warning("Overwriting the previous mean offset and zero-mode")
        self._offset_mean = offset_mean
        self._offset_std = None
        if offset_std is None:
            self._azm = 0.
        elif np.isscalar(offset_std) and offset_std == 1.:
            self._azm = 1.
        elif isinstance(offset_std, Operator):
            self._azm = offset_std
        else:
            if dofdex is not None and len(dofdex) != self._total_N:
                raise ValueError("length of dofdex needs to match total_N")
            if len(offset_std) != 2:
                raise TypeError("`offset_std` of invalid type and/or shape; expected a 2D tuple "
                                f"of floats; got '{offset_std!r}'")
            self._offset_std = tuple(offset_std)
            self._azm = LognormalTransform(*offset_std, self._prefix + 'zeromode', 0)

    # ------------------------------------------------------------ lowering
    def _fusable(self):
        """One non-parametric component on an RGSpace, zero mode off or
        LogNormal: the case the fused operator restates exactly."""
        if len(self._a) != 1 or not hasattr(self._a[0], "model"):
            return False
        if not (self._azm is not None and (self._offset_std is not None
                                           or (np.isscalar(self._azm) and self._azm == 0))):
            return False
        tgt = self._target_subdomains[0]
        return len(tgt) == 1 and _rg_only(tgt) and _rg_only((self._a[0].harmonic_partner,))

    def _fused_model(self, offset_mean):
        from .correlated_fields_simple import _CorrelatedFieldModel
        a = self._a[0]
        fl, flex, asp, slope, pre = a.params
        return _CorrelatedFieldModel(self._target_subdomains[0][0], a.harmonic_partner, offset_mean,
                                     self._offset_std, fl, flex, asp, slope, pre, xi_prefix=self._prefix)

    def finalize(self, prior_info=100):
        """(correlated_fields.py:764-823)"""
        from functools import reduce
        from operator import mul
        from ..multi_field import MultiField
        from ..operators.adder import Adder
        from ..operators.contraction_operator import ContractionOperator
        from ..operators.distributors import PowerDistributor
        from ..operators.harmonic_operators import HarmonicTransformOperator
        from ..operators.simple_linear_operators import ducktape
        from ..sugar import full
        om = self._offset_mean
        if self._fusable() and (om is None or np.isscalar(om)):
            op = self._fused_model(None if om is None else float(om))
            self.statistics_summary(prior_info)
            return op
        n_amplitudes = len(self._a)
        hspace = makeDomain([dd.target[0].harmonic_partner for dd in self._a])
        spaces = tuple(range(n_amplitudes))
        ht = HarmonicTransformOperator(hspace, self._target_subdomains[0][0], space=spaces[0])
        for i in range(1, n_amplitudes):
            ht = HarmonicTransformOperator(ht.target, self._target_subdomains[i][0], space=spaces[i]) @ ht
        a = list(self.get_normalized_amplitudes())
        for ii in range(n_amplitudes):
            co = ContractionOperator(hspace, spaces[:ii] + spaces[ii + 1:])
            pd = PowerDistributor(co.target, a[ii].target[0], 0)
            a[ii] = co.adjoint @ pd @ a[ii]
        corr = reduce(mul, a)
        xi = ducktape(hspace, None, self._prefix + 'xi')
        if np.isscalar(self.azm):
            op = ht(corr * xi)
        else:
            expander = ContractionOperator(hspace, spaces=spaces).adjoint
            op = ht((expander @ self.azm) * corr * xi)
        if om is not None:
            if isinstance(om, (Field, MultiField)):
                op = Adder(om) @ op
            else:
                op = Adder(full(op.target, float(om))) @ op
        self.statistics_summary(prior_info)
        return op

    def statistics_summary(self, prior_info):
        """(correlated_fields.py:825-856)"""
        from ..logger import logger
        from ..probing import StatCalculator
        from ..sugar import from_random
        if prior_info == 0:
            return
        lst = []
        try:
            lst.append(('Offset amplitude', self.amplitude_total_offset))
        except NotImplementedError:
            pass
        lst.append(('Total fluctuation amplitude', self.total_fluctuation))
        namps = len(self._a)
        if namps > 1:
            for ii in range(namps):
                lst.append((f'Average fluctuation (space {ii})', self.average_fluctuation(ii)))
                try:
                    lst.append((f'Slice fluctuation (space {ii})', self.slice_fluctuation(ii)))
                except NotImplementedError:
                    pass
        for kk, op in lst:
            if np.isscalar(op):
                continue
            sc = StatCalculator()
            for _ in range(prior_info):
                sc.add(op(from_random(op.domain, 'normal')))
            mean = np.asarray(sc.mean.val_np())
            stddev = np.asarray(sc.var.ptw("sqrt").val_np())
            for m, s in zip(mean.flatten(), stddev.flatten()):
                logger.info('{}: {:.02E} ± {:.02E}'.format(kk, m, s))

    @property
    def fluctuations(self):
        return tuple(self._a)

    def get_normalized_amplitudes(self):
        """(correlated_fields.py:862-917)"""
        from ..operators.adder import Adder
        from ..operators.contraction_operator import ContractionOperator
        from ..operators.diagonal_operator import DiagonalOperator
        from ..sugar import full, makeField, makeOp
        if self._azm == 0:
            if not len(self.fluctuations) == 1:
                raise RuntimeError("Zeromode can not be disabled for product spectra")
            sp = self.fluctuations[0].target
            maskzm = np.ones(sp.shape)
            maskzm[0] = 0
            return (makeOp(makeField(sp, maskzm)) @ self.fluctuations[0],)
        elif np.isscalar(self.azm) and self.azm == 1:
            return self.fluctuations
        normal_amp = []
        for amp in self._a:
            a_target = amp.target
            a_space = getattr(amp, "_space", 0)
            a_pp = amp.target[a_space]
            myassert(isinstance(a_pp, PowerSpace))
            azm_expander = ContractionOperator(a_target, spaces=a_space).adjoint
            zm_unmask, zm_mask = np.zeros(a_pp.shape), np.zeros(a_pp.shape)
            zm_mask[1:] = zm_unmask[0] = 1.
            zm_mask = DiagonalOperator(makeField(a_pp, zm_mask), a_target, a_space)
            zm_unmask = DiagonalOperator(makeField(a_pp, zm_unmask), a_target, a_space)
            zm_unmask = Adder(zm_unmask(full(zm_unmask.domain, 1)))
            zm_normalization = zm_unmask @ (zm_mask @ azm_expander(self.azm.ptw("reciprocal")))
            normal_amp.append(zm_normalization * amp)
        return tuple(normal_amp)

    @property
    def amplitude(self):
        """(correlated_fields.py:919-938); the fused amplitude operator for
        the single-component case `finalize` lowers to the fused field."""
        from ..operators.contraction_operator import ContractionOperator
        if len(self._a) > 1:
            raise NotImplementedError(
                'If more than one spectrum is present in the model, no unique set of amplitudes '
                'exist because only the relative scale is determined.')
        if self._fusable():
            return self._fused_model(None).amplitude
        normal_amp = self.get_normalized_amplitudes()[0]
        if np.isscalar(self.azm):
            return normal_amp
        expand = ContractionOperator(normal_amp.target, len(normal_amp.target) - 1).adjoint
        return normal_amp * (expand @ self.azm)

    @property
    def power_spectrum(self):
        return self.amplitude ** 2

    @property
    def amplitude_total_offset(self):
        if self._azm is None:
            raise NotImplementedError("You need to set the `amplitude_total_offset` first")
        return self._azm

    @property
    def azm(self):
        return self.amplitude_total_offset

    def moment_slice_to_average(self, fluctuations_slice_mean, nsamples=1000):
        """(correlated_fields.py:948-1007)"""
        from ..sugar import from_random
        fluctuations_slice_mean = float(fluctuations_slice_mean)
        if not fluctuations_slice_mean > 0:
            raise ValueError(f"fluctuations_slice_mean must be greater zero; got {fluctuations_slice_mean!r}")
        scm = 1.
        for a in self._a:
            op = a.fluctuation_amplitude * self.azm.ptw("reciprocal")
            res = np.array([op(from_random(op.domain, 'normal')).val_np() for _ in range(nsamples)])
            scm *= res ** 2 + 1.
        return fluctuations_slice_mean / np.mean(np.sqrt(scm))

    @property
    def total_fluctuation(self):
        """(correlated_fields.py:1009-1020)"""
        from ..operators.adder import Adder
        from ..sugar import full
        if len(self._a) == 0:
            raise NotImplementedError
        if len(self._a) == 1:
            return self.average_fluctuation(0)
        q = 1.
        for a in self._a:
            fl = a.fluctuation_amplitude * self.azm.ptw("reciprocal")
            q = q * (Adder(full(fl.target, 1.)) @ fl ** 2)
        return (Adder(full(q.target, -1.)) @ q).ptw("sqrt") * self.azm

    def slice_fluctuation(self, space):
        """(correlated_fields.py:1022-1037)"""
        from ..operators.adder import Adder
        from ..sugar import full
        if len(self._a) == 0:
            raise NotImplementedError
        if space >= len(self._a):
            raise ValueError(f"invalid space specified; got {space!r}")
        if len(self._a) == 1:
            return self.average_fluctuation(0)
        q = 1.
        for j in range(len(self._a)):
            fl = self._a[j].fluctuation_amplitude * self.azm.ptw("reciprocal")
            if j == space:
                q = q * fl ** 2
            else:
                q = q * (Adder(full(fl.target, 1.)) @ fl ** 2)
        return q.ptw("sqrt") * self.azm

    def average_fluctuation(self, space):
        """(correlated_fields.py:1039-1048)"""
        if len(self._a) == 0:
            raise NotImplementedError
        if space >= len(self._a):
            raise ValueError(f"invalid space specified; got {space!r}")
        if len(self._a) == 1:
            return self._a[0].fluctuation_amplitude
        return self._a[space].fluctuation_amplitude

    @staticmethod
    def offset_amplitude_realized(samples):
        """(correlated_fields.py:1050-1057)"""
        spaces = _structured_spaces(samples[0].domain)
        res = 0.
        for s in samples:
            res = res + s.mean(spaces) ** 2
        res = res / len(samples)
        return np.sqrt(res if np.isscalar(res) else res.val_np())

    @staticmethod
    def total_fluctuation_realized(samples):
        return _total_fluctuation_realized(samples)

    @staticmethod
    def slice_fluctuation_realized(samples, space):
        """(correlated_fields.py:1063-1083)"""
        spaces = _structured_spaces(samples[0].domain)
        if space >= len(spaces):
            raise ValueError(f"invalid space specified; got {space!r}")
        if len(spaces) == 1:
            return _total_fluctuation_realized(samples)
        space = space + spaces[0]
        res1, res2 = 0., 0.
        for s in samples:
            res1 = res1 + s ** 2
            res2 = res2 + s.mean(space) ** 2
        res1 = res1 / len(samples)
        res2 = res2 / len(samples)
        res = res1.mean(tuple(spaces)) - res2.mean(tuple(spaces[:-1]))
        return np.sqrt(res if np.isscalar(res) else res.val_np())

    @staticmethod
    def average_fluctuation_realized(samples, space):
        """(correlated_fields.py:1085-1109)"""
        from ..operators.contraction_operator import ContractionOperator
        spaces = _structured_spaces(samples[0].domain)
        if space >= len(spaces):
            raise ValueError(f"invalid space specified; got {space!r}")
        if len(spaces) == 1:
            return _total_fluctuation_realized(samples)
        space = space + spaces[0]
        sub_spaces = set(int(s) for s in spaces)
        sub_spaces.remove(space)
        sub_dom = makeDomain([samples[0].domain[ind]
                              for ind in (set([0]) - set(int(s) for s in spaces)) | set([space])])
        co = ContractionOperator(sub_dom, len(sub_dom) - 1)
        size = co.domain.size / co.target.size
        res = 0.
        for s in samples:
            r = s.mean(tuple(sorted(sub_spaces)))
            res = res + (r - co.adjoint(co(r) / size)) ** 2
        res = res.mean(int(spaces[0])) / len(samples)
        return np.sqrt(res if np.isscalar(res) else res.val_np())
