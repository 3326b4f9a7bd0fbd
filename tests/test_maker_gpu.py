"""CorrelatedFieldMaker (src/library/correlated_fields.py:388-1115) on the
device: the single-component lowering to the fused SimpleCorrelatedField
operator (test_complicated_vs_simple, test/test_operators/
test_correlated_fields.py:214-272), the reference's operator tree for product
spectra / unit zero mode / Matern against the reference's own outputs
(tests/golden/cfm.npz from gen_golden.py:gen_cfm), and the zero-mode
invariants of test_unit_zero_mode / test_constant_zero_mode (:88-148).

Tolerances (fp64): values, Jacobians and adjoints rtol 1e-10 (two FFT engines
and two summation orders apart); fused vs operator tree 1e-11."""
import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a)
    b = np.asarray(b)
    nb = np.linalg.norm(b)
    return np.linalg.norm(a - b) / (nb if nb > 0 else 1.)


@pytest.fixture(scope="module")
def ift(dev):
    import nifty_amd
    return nifty_amd


def _mf(ift, dom, G, prefix):
    return ift.MultiField.from_dict({k: ift.makeField(dom[k], G[prefix + k]) for k in dom.keys()}, dom)


def _rand_mf(ift, dom, seed):
    rng = np.random.default_rng(seed)
    return ift.MultiField.from_dict({k: ift.makeField(dom[k], rng.standard_normal(dom[k].shape))
                                     for k in dom.keys()}, dom)


def _lin(ift, op, x):
    return op(ift.Linearization.make_var(x))


def _vdot(a, b):
    if hasattr(a, "keys"):
        return sum(float(torch.sum(a[k].val * b[k].val)) for k in a.keys())
    return float(torch.sum(a.val * b.val))


# ------------------------------------------------- complicated vs simple
def _posrand(rng):
    return float(np.exp(rng.standard_normal()))


@pytest.mark.parametrize("seed", [13, 2])
@pytest.mark.parametrize("shape,dist", [((12,), None), ((13,), 0.7), ((14, 15), (0.3, 1.2)), ((9, 8, 6), None)])
@pytest.mark.parametrize("without", [(), ("offset_std",), ("asperity",), ("flexibility",),
                                     ("flexibility", "asperity"), ("offset_std", "flexibility", "asperity")])
def test_complicated_vs_simple(ift, seed, shape, dist, without):
    """(test_correlated_fields.py:214-272): the Maker with one component is
    the fused SimpleCorrelatedField -- same domain object, same values and
    amplitude -- and the reference's generic operator tree built from the
    same Maker (lowering disabled) agrees with it in value and Jacobian."""
    from nifty_amd.library.correlated_fields_simple import _CorrelatedFieldModel
    rng = np.random.default_rng(seed)
    domain = ift.RGSpace(shape, distances=dist)
    offset_mean = float(rng.standard_normal())
    fluctuations = _posrand(rng), _posrand(rng)
    flexibility = None if "flexibility" in without else (_posrand(rng), _posrand(rng))
    asperity = None if "asperity" in without else (_posrand(rng), _posrand(rng))
    offset_std = None if "offset_std" in without else (_posrand(rng), _posrand(rng))
    loglogavgslope = _posrand(rng), _posrand(rng)
    prefix = 'foobar'
    hspace = domain.get_default_codomain()
    cfm = ift.CorrelatedFieldMaker(prefix)
    if asperity is not None and flexibility is None:
        with pytest.raises(ValueError):
            ift.SimpleCorrelatedField(domain, offset_mean, offset_std, fluctuations, flexibility, asperity,
                                      loglogavgslope, prefix=prefix, harmonic_partner=hspace)
        with pytest.raises(ValueError):
            cfm.add_fluctuations(domain, fluctuations, flexibility, asperity, loglogavgslope, prefix='',
                                 harmonic_partner=hspace)
        return
    scf = ift.SimpleCorrelatedField(domain, offset_mean, offset_std, fluctuations, flexibility, asperity,
                                    loglogavgslope, prefix=prefix, harmonic_partner=hspace)
    cfm.add_fluctuations(domain, fluctuations, flexibility, asperity, loglogavgslope, prefix='',
                         harmonic_partner=hspace)
    cfm.set_amplitude_total_offset(offset_mean, offset_std)
    inp = _rand_mf(ift, scf.domain, seed + 100)
    op1 = cfm.finalize(prior_info=0)
    assert isinstance(op1, _CorrelatedFieldModel)
    assert scf.domain is op1.domain
    assert rel(op1(inp).val, scf(inp).val.cpu().numpy()) < 1e-14
    a1, a0 = cfm.amplitude, scf.amplitude
    assert a0.domain is a1.domain
    assert rel(a1.force(inp).val, a0.force(inp).val.cpu().numpy()) < 1e-14

    # the reference's operator tree from the same maker
    cfm._fusable = lambda: False
    tree = cfm.finalize(prior_info=0)
    assert not isinstance(tree, _CorrelatedFieldModel)
    assert tree.domain is scf.domain
    lf, lt = _lin(ift, scf, inp), _lin(ift, tree, inp)
    assert rel(lt.val.val, lf.val.val.cpu().numpy()) < 1e-11
    t = _rand_mf(ift, scf.domain, seed + 200)
    assert rel(lt.jac(t).val, lf.jac(t).val.cpu().numpy()) < 1e-11
    g = ift.makeField(scf.target, np.random.default_rng(seed + 300).standard_normal(scf.target.shape))
    jf, jt = lf.jac.adjoint(g), lt.jac.adjoint(g)
    for k in scf.domain.keys():
        assert rel(jt[k].val, jf[k].val.cpu().numpy()) < 1e-11, k
    at = cfm.amplitude
    assert rel(at.force(inp).val, a0.force(inp).val.cpu().numpy()) < 1e-13


# --------------------------------------------------------- golden (cfm.npz)
def _maker(ift, tag):
    """the makers of gen_golden.py:gen_cfm"""
    if tag == "prod_":
        cfm = ift.CorrelatedFieldMaker("pp_")
        cfm.add_fluctuations(ift.RGSpace((24, 20), distances=(0.05, 0.07)), (1., 0.4), (1.2, 0.5), (0.6, 0.3),
                             (-3., 0.5), prefix="sp_")
        cfm.add_fluctuations(ift.RGSpace(18, distances=0.3), (0.7, 0.2), (0.9, 0.4), None, (-2., 0.4),
                             prefix="fr_")
        cfm.set_amplitude_total_offset(0.3, (0.8, 0.1))
    elif tag == "one_":
        cfm = ift.CorrelatedFieldMaker("mk_")
        cfm.add_fluctuations(ift.RGSpace((40, 36), distances=(0.02, 0.03)), (0.9, 0.3), (1.1, 0.4), (0.5, 0.2),
                             (-2.5, 0.6), prefix="amp_")
        cfm.set_amplitude_total_offset(-0.4, (1e-2, 1e-3))
    elif tag == "unit_":
        cfm = ift.CorrelatedFieldMaker("u_")
        cfm.add_fluctuations(ift.RGSpace(64), (1., 0.5), None, None, (-3., 1.))
        cfm.set_amplitude_total_offset(0., 1.)
    else:
        cfm = ift.CorrelatedFieldMaker("m_")
        cfm.add_fluctuations_matern(ift.RGSpace((32, 32), distances=0.1), (1., 0.3), (2., 0.5), (-3., 0.5))
        cfm.set_amplitude_total_offset(1., (1e-2, 1e-3))
    return cfm


@pytest.mark.parametrize("tag", ["prod_", "one_", "unit_", "mat_"])
def test_maker_golden(ift, tag):
    """value, J t and J^T g of the finalized operator, and the (normalised)
    amplitudes, against the reference's (gen_golden.py:gen_cfm)."""
    from nifty_amd.library.correlated_fields_simple import _CorrelatedFieldModel
    G = golden("cfm.npz")
    cfm = _maker(ift, tag)
    op = cfm.finalize(prior_info=0)
    assert isinstance(op, _CorrelatedFieldModel) == (tag == "one_")
    keys = sorted(k[len(tag) + 2:] for k in G.files if k.startswith(tag + "x_"))
    assert sorted(op.domain.keys()) == keys
    x, t = _mf(ift, op.domain, G, tag + "x_"), _mf(ift, op.domain, G, tag + "t_")
    lin = _lin(ift, op, x)
    assert rel(lin.val.val, G[tag + "val"]) < 1e-10
    assert rel(lin.jac(t).val, G[tag + "jt"]) < 1e-10
    ja = lin.jac.adjoint(ift.makeField(op.target, G[tag + "g"]))
    for k in keys:
        assert rel(ja[k].val, G[tag + "ja_" + k]) < 1e-10, k
    if tag == "prod_":
        for i, na in enumerate(cfm.get_normalized_amplitudes()):
            assert rel(na.force(x).val, G[f"prod_na{i}"]) < 1e-10
        assert rel(cfm.total_fluctuation.force(x).val, G["prod_totfl"]) < 1e-12
        for i in range(2):
            assert rel(cfm.slice_fluctuation(i).force(x).val, G[f"prod_slfl{i}"]) < 1e-12
            assert rel(cfm.average_fluctuation(i).force(x).val, G[f"prod_avfl{i}"]) < 1e-12
        with pytest.raises(NotImplementedError):
            cfm.amplitude
    else:
        assert rel(cfm.amplitude.force(x).val, G[tag + "amp"]) < 1e-10


# ------------------------------------------------------- zero-mode invariants
@pytest.mark.parametrize("shape", [(10,), (7, 8)])
@pytest.mark.parametrize("flex_asp", [(None, None), ((1, 1), None), ((1, 1), (1, 1))])
@pytest.mark.parametrize("matern", [False, True])
def test_unit_and_constant_zero_mode(ift, shape, flex_asp, matern):
    """(test_correlated_fields.py:88-148): unit zero mode with xi[0] = 1
    integrates to the total volume; a disabled zero mode integrates to 0."""
    sspace = ift.RGSpace(shape, distances=0.3)
    flexibility, asperity = flex_asp
    cfg = 1, 1
    cfm = ift.CorrelatedFieldMaker('')
    if matern:
        cfm.add_fluctuations_matern(sspace, *(3 * [cfg]))
    else:
        cfm.add_fluctuations(sspace, cfg, flexibility, asperity, cfg)
    cfm.set_amplitude_total_offset(0, 1.)
    cf = cfm.finalize(prior_info=0)
    r = _rand_mf(ift, cf.domain, 7).to_dict()
    xi = r["xi"].val.clone()
    xi.view(-1)[0] = 1.
    r["xi"] = ift.Field(r["xi"].domain, xi)
    r = ift.MultiField.from_dict(r)
    np.testing.assert_allclose(float(cf(r).s_integrate()), sspace.total_volume, rtol=1e-7)

    cfm = ift.CorrelatedFieldMaker('')
    if matern:
        cfm.add_fluctuations_matern(sspace, *(3 * [cfg]))
    else:
        cfm.add_fluctuations(sspace, (1., 0.5), flexibility, asperity, (-4, 1))
    cfm.set_amplitude_total_offset(0, None)
    cf = cfm.finalize(prior_info=0)
    r = _rand_mf(ift, cf.domain, 8)
    np.testing.assert_allclose(float(cf(r).s_integrate()), 0., atol=1e-8)


def _stats(ift, op, samples):
    sc = ift.StatCalculator()
    for s in samples:
        sc.add(op(s.extract(op.domain)))
    return sc.mean.val_np(), sc.var.ptw("sqrt").val_np()


@pytest.mark.parametrize("sshape", [(8,), (12, 10)])
def test_amplitudes_invariants(ift, sshape):
    """testAmplitudesInvariants (test_correlated_fields.py:147-210, N = 0):
    the prior statistics of total / average / slice fluctuation and offset
    operators agree with the *_realized estimates on field samples, and
    moment_slice_to_average recovers the slice fluctuation."""
    sspace = ift.RGSpace(sshape, distances=0.3)
    fsspace = ift.RGSpace((12,), (0.4,))
    astds = 0.2, 1.2
    offset_std_mean = 1.3
    fa = ift.CorrelatedFieldMaker('')
    fa.add_fluctuations(sspace, (astds[0], 1e-2), (1.1, 2.), (2.1, .5), (-2, 1.), 'spatial')
    fa.add_fluctuations(fsspace, (astds[1], 1e-2), (3.1, 1.), (.5, .1), (-4, 1.), 'freq')
    fa.set_amplitude_total_offset(1.2, (offset_std_mean, 1e-2))
    op = fa.finalize(prior_info=2)
    samples = [_rand_mf(ift, op.domain, 500 + i) for i in range(100)]
    tot_flm, _ = _stats(ift, fa.total_fluctuation, samples)
    offset_amp_std, _ = _stats(ift, fa.amplitude_total_offset, samples)
    fl0, _ = _stats(ift, fa.average_fluctuation(0), samples)
    fl1, _ = _stats(ift, fa.average_fluctuation(1), samples)
    sl0, _ = _stats(ift, fa.slice_fluctuation(0), samples)
    sl1, _ = _stats(ift, fa.slice_fluctuation(1), samples)
    sams = [op(s) for s in samples]
    np.testing.assert_allclose(offset_amp_std, fa.offset_amplitude_realized(sams), rtol=0.5)
    np.testing.assert_allclose(fl0, fa.average_fluctuation_realized(sams, 0), rtol=0.5)
    np.testing.assert_allclose(fl1, fa.average_fluctuation_realized(sams, 1), rtol=0.5)
    np.testing.assert_allclose(tot_flm, fa.total_fluctuation_realized(sams), rtol=0.5)
    np.testing.assert_allclose(sl0, fa.slice_fluctuation_realized(sams, 0), rtol=0.5)
    np.testing.assert_allclose(sl1, fa.slice_fluctuation_realized(sams, 1), rtol=0.5)

    fa = ift.CorrelatedFieldMaker('')
    fa.set_amplitude_total_offset(0., (offset_std_mean, .1))
    fa.add_fluctuations(fsspace, (astds[1], 1.), (3.1, 1.), (.5, .1), (-4, 1.), 'freq')
    m = 3.
    x = fa.moment_slice_to_average(m, nsamples=300)
    fa.add_fluctuations(sspace, (x, 1.5), (1.1, 2.), (2.1, .5), (-2, 1.), 'spatial', 0)
    op = fa.finalize(prior_info=0)
    em, _ = _stats(ift, fa.slice_fluctuation(0), samples)
    np.testing.assert_allclose(m, em, rtol=0.5)
    assert op.target[-2] == sspace
    assert op.target[-1] == fsspace
    # Jacobian consistency of the normalised amplitudes and the field
    for ampl in list(fa.get_normalized_amplitudes()) + [op]:
        x0 = _rand_mf(ift, ampl.domain, 9)
        x0 = ift.MultiField.from_dict({k: x0[k] * 0.1 for k in x0.keys()})
        lin = _lin(ift, ampl, x0)
        t = _rand_mf(ift, ampl.domain, 10)
        g = ift.makeField(ampl.target, np.random.default_rng(11).standard_normal(ampl.target.shape))
        lhs = _vdot(lin.jac(t), g)
        rhs = _vdot(t, lin.jac.adjoint(g))
        assert abs(lhs - rhs) <= 1e-10 * max(abs(lhs), 1.)
        eps = 1e-6
        xp = ift.MultiField.from_dict({k: x0[k] + t[k] * eps for k in x0.keys()})
        xm = ift.MultiField.from_dict({k: x0[k] - t[k] * eps for k in x0.keys()})
        fd = (ampl(xp).val - ampl(xm).val) / (2 * eps)
        jt = lin.jac(t).val
        assert float(torch.linalg.norm(fd - jt)) <= 1e-5 * max(float(torch.linalg.norm(jt)), 1e-3)
