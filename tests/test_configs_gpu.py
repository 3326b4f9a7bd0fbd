"""BASELINE.json configs C2-C5 at full size on one MI355X, checked through
size-independent properties (the oracle does not finish at these sizes in
seconds; the small-size parity against the reference's golden vectors is in
test_parity_gpu.py):

  C2  1024^2 CorrelatedField + Poisson, geoVI n_samples=4 (8 mirrored)
  C3  2048^2 LOSResponse(16384) + sigmoid + Gaussian (the bench workload)
  C4  512^3 3-D CorrelatedField + GeometryRemover Gaussian
  C5  4096^2 CorrelatedField + Gaussian

Properties: symmetry of the sampling metric <u, M v> = <M u, v> and its
positivity, adjointness of the LOS box kernels and of the CF Jacobian,
Hartley round trips, CG energy decrease, mirrored-sample structure and
finiteness of a full geoVI draw (C2)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

CF_ARGS = dict(offset_mean=0, offset_std=(1e-3, 1e-6), fluctuations=(1., 0.8),
               loglogavgslope=(-3., 1), flexibility=(2, 1.), asperity=(0.5, 0.4))


@pytest.fixture(scope="module")
def ift(dev):
    import nifty_amd
    return nifty_amd


def _dot(a, b):
    return sum(float(torch.sum(a[k].val * b[k].val)) for k in a.keys())


def _metric(ift, lh, pos):
    dtype, f_lh = lh.get_transformation()
    fl = f_lh(ift.Linearization.make_var(pos))
    return (ift.SandwichOperator.make(fl.jac, ift.ScalingOperator(f_lh.target, 1., dtype))
            + ift.ScalingOperator(fl.domain, 1., float)), fl


def _check_metric(ift, met, dom, tol=1e-10):
    u = ift.from_random(dom, "normal")
    v = ift.from_random(dom, "normal")
    mu, mv = met(u), met(v)
    a, b = _dot(u, mv), _dot(mu, v)
    assert abs(a - b) <= tol * max(abs(a), abs(b)), (a, b)
    assert _dot(u, mu) >= _dot(u, u) * (1 - 1e-12)   # M = 1 + J^T W J >= 1


def _gauss_problem(ift, shape, var=0.01, seed=17):
    sp = ift.RGSpace(shape)
    cf = ift.SimpleCorrelatedField(sp, **dict(CF_ARGS, asperity=None) if len(shape) == 3 else CF_ARGS)
    R = ift.GeometryRemover(sp)
    ift.random.push_sseq_from_seed(seed)
    N = ift.ScalingOperator(R.target, var, np.float64)
    data = R(cf(ift.from_random(cf.domain, "normal"))) + N.draw_sample()
    pos = 0.1 * ift.from_random(cf.domain, "normal")
    ift.random.pop_sseq()
    lh = ift.GaussianEnergy(data, inverse_covariance=N.inverse) @ (R @ cf)
    return cf, lh, pos


def test_c2_poisson_geovi_1024(ift):
    sp = ift.RGSpace((1024, 1024))
    cf = ift.SimpleCorrelatedField(sp, **CF_ARGS)
    sig = cf.exp()
    ift.random.push_sseq_from_seed(27)
    lam = sig(ift.from_random(cf.domain, "normal")).val.cpu().numpy()
    counts = ift.random.current_rng().poisson(lam).astype(np.int64)
    pos = 0.1 * ift.from_random(cf.domain, "normal")
    ift.random.pop_sseq()
    lh = ift.PoissonianEnergy(ift.makeField(sp, counts)) @ sig
    met, _ = _metric(ift, lh, pos)
    ift.random.push_sseq_from_seed(1)
    _check_metric(ift, met, cf.domain)
    ift.random.pop_sseq()
    H = ift.StandardHamiltonian(lh, ift.GradientNormController(iteration_limit=20))
    mini = ift.NewtonCG(ift.GradientNormController(iteration_limit=2), max_cg_iterations=10)
    ift.random.push_sseq_from_seed(5)
    sl = ift.draw_samples(pos, H, mini, 4, True)
    ift.random.pop_sseq()
    assert sl.n_samples == 8
    for r in sl._r:
        for k in cf.domain.keys():
            assert torch.isfinite(r[k].val).all()
    kl = ift.SampledKLEnergyClass(sl, H, [], None, True)
    assert np.isfinite(kl.value)


def test_c3_los_2048_adjoint_and_metric(ift):
    sp = ift.RGSpace((2048, 2048))
    cf = ift.SimpleCorrelatedField(sp, **CF_ARGS)
    ift.random.push_sseq_from_seed(27)
    rng = ift.random.current_rng()
    nlos = 16384
    starts = list(rng.random((nlos, 2)).T)
    ends = list(rng.random((nlos, 2)).T)
    R = ift.LOSResponse(sp, starts=starts, ends=ends)
    x = ift.from_random(R.domain, "normal")
    y = ift.from_random(R.target, "normal")
    a = float(torch.sum(R(x).val * y.val))
    b = float(torch.sum(x.val * R.adjoint(y).val))
    assert abs(a - b) <= 1e-11 * abs(a)
    sr = R @ ift.sigmoid(cf)
    N = ift.ScalingOperator(R.target, 1e-3, np.float64)
    data = sr(ift.from_random(cf.domain, "normal")) + N.draw_sample()
    pos = 0.1 * ift.from_random(cf.domain, "normal")
    lh = ift.GaussianEnergy(data, inverse_covariance=N.inverse) @ sr
    met, fl = _metric(ift, lh, pos)
    _check_metric(ift, met, cf.domain)
    # CF Jacobian adjointness at full size
    u = ift.from_random(cf.domain, "normal")
    g = ift.from_random(fl.target, "normal")
    a = float(torch.sum(fl.jac(u).val * g.val))
    b = _dot(u, fl.jac.adjoint(g))
    assert abs(a - b) <= 1e-10 * abs(a)
    ift.random.pop_sseq()


def test_c4_cube_512(ift):
    shape = (512, 512, 512)
    sp = ift.RGSpace(shape)
    ht = ift.HartleyOperator(sp.get_default_codomain(), sp)
    ift.random.push_sseq_from_seed(2)
    x = ift.Field(ht.domain, torch.randn(shape, dtype=torch.float64, device="cuda"))
    y = ht.inverse_times(ht.times(x))
    err = float(torch.linalg.vector_norm(y.val - x.val) / torch.linalg.vector_norm(x.val))
    assert err < 1e-12
    del y
    cf, lh, pos = _gauss_problem(ift, shape)
    met, _ = _metric(ift, lh, pos)
    _check_metric(ift, met, cf.domain)
    b = ift.from_random(cf.domain, "normal")
    ic = ift.GradientNormController(iteration_limit=3)
    en, st = ift.ConjugateGradient(ic)(ift.QuadraticEnergy(0 * b, met, b))
    assert st == ic.CONVERGED and en.value < 0
    ift.random.pop_sseq()


def test_c5_4096(ift):
    cf, lh, pos = _gauss_problem(ift, (4096, 4096))
    met, _ = _metric(ift, lh, pos)
    ift.random.push_sseq_from_seed(9)
    _check_metric(ift, met, cf.domain)
    b = ift.from_random(cf.domain, "normal")
    ic = ift.GradientNormController(iteration_limit=3)
    en, st = ift.ConjugateGradient(ic)(ift.QuadraticEnergy(0 * b, met, b))
    assert st == ic.CONVERGED and en.value < 0
    ift.random.pop_sseq()


@pytest.mark.parametrize("shape", [(256, 256), (4096, 4096), "los"])
def test_c5_fp32_mixed_precision_cg(ift, shape):
    """C5's fp32 storage / fp64-accumulated CG (config.set_cg_precision("fp32"))
    against the fp64 solve of the same system: rtol 1e-4 (BASELINE.json C5)."""
    from nifty_amd import config
    from nifty_amd.minimization.fused_cg import fusable_metric, mixed_precision
    if shape == "los":
        sp = ift.RGSpace((512, 512))
        cf = ift.SimpleCorrelatedField(sp, **CF_ARGS)
        ift.random.push_sseq_from_seed(8)
        rng = ift.random.current_rng()
        R = ift.LOSResponse(sp, starts=list(rng.random((2000, 2)).T), ends=list(rng.random((2000, 2)).T))
        sr = R @ ift.sigmoid(cf)
        N = ift.ScalingOperator(R.target, 1e-3, np.float64)
        data = sr(ift.from_random(cf.domain, "normal")) + N.draw_sample()
        pos = 0.1 * ift.from_random(cf.domain, "normal")
        ift.random.pop_sseq()
        lh = ift.GaussianEnergy(data, inverse_covariance=N.inverse) @ sr
    else:
        cf, lh, pos = _gauss_problem(ift, shape)
    met, _ = _metric(ift, lh, pos)
    config.set_cg_precision("fp32")
    try:
        core, W, _ = fusable_metric(met)
        assert mixed_precision(core, W)   # the fp32 pipeline is the one that runs
    finally:
        config.set_cg_precision("fp64")
    ift.random.push_sseq_from_seed(4)
    b = ift.from_random(cf.domain, "normal")
    ift.random.pop_sseq()
    res = {}
    for prec in ("fp64", "fp32"):
        config.set_cg_precision(prec)
        try:
            ic = ift.GradientNormController(iteration_limit=8)
            en, st = ift.ConjugateGradient(ic)(ift.QuadraticEnergy(0 * b, met, b))
        finally:
            config.set_cg_precision("fp64")
        assert st == ic.CONVERGED
        res[prec] = en
    for k in cf.domain.keys():
        a = res["fp32"].position[k].val
        r = res["fp64"].position[k].val
        assert a.dtype == torch.float64
        err = float(torch.linalg.vector_norm(a - r) / torch.linalg.vector_norm(r))
        assert err < 1e-4, (k, err)
    assert abs(res["fp32"].value - res["fp64"].value) < 1e-4 * abs(res["fp64"].value)


def _kl_checks(ift, sl, H, n):
    assert sl.n_samples == n and len(sl._r) == n
    for r in sl._r:
        for k in r.keys():
            assert bool(torch.all(torch.isfinite(r[k].val))), k
    kl = ift.SampledKLEnergyClass(sl, H, [], None, True)
    assert np.isfinite(kl.value)
    for k in kl.gradient.keys():
        assert bool(torch.all(torch.isfinite(kl.gradient[k].val))), k
    return kl


def test_c4_geovi_draw_512(ift):
    """C4's per-GPU share (n_samples=16 mirrored over 8 GPUs: 2 pairs) as a
    geoVI draw at 512^3: linear CG 10 steps, one Newton step (inner CG 5),
    batched refinement of the 4 samples; finite samples, the two members of a
    pair start mirrored about the expansion point, finite KL value and
    gradient."""
    cf, lh, pos = _gauss_problem(ift, (512, 512, 512))
    H = ift.StandardHamiltonian(lh, ift.GradientNormController(iteration_limit=10))
    mini = ift.NewtonCG(ift.GradientNormController(iteration_limit=1))
    ift.random.push_sseq_from_seed(12)
    sl = ift.draw_samples(pos, H, mini, 2, True)
    ift.random.pop_sseq()
    _kl_checks(ift, sl, H, 4)
    # the refinement moves the mirrored starts only a little: the pair stays
    # roughly antisymmetric about the expansion point
    for a, b in ((0, 1), (2, 3)):
        ra, rb = sl._r[a]["xi"].val, sl._r[b]["xi"].val
        asym = float(torch.linalg.vector_norm(ra + rb) / torch.linalg.vector_norm(ra - rb))
        assert asym < 0.5, asym


def test_c5_geovi_draw_4096_fp32(ift):
    """C5's per-GPU share (n_samples=32 mirrored over 8 GPUs: 4 pairs) as a
    geoVI draw at 4096^2 with fp32 CG storage (config.set_cg_precision("fp32"),
    fp64 reductions): finite samples and KL, and every sample within rtol
    1e-4 of the same draw in fp64 (BASELINE.json C5)."""
    from nifty_amd import config
    cf, lh, pos = _gauss_problem(ift, (4096, 4096))
    H = ift.StandardHamiltonian(lh, ift.GradientNormController(iteration_limit=8))
    out = {}
    for prec in ("fp64", "fp32"):
        config.set_cg_precision(prec)
        try:
            mini = ift.NewtonCG(ift.GradientNormController(iteration_limit=1))
            ift.random.push_sseq_from_seed(13)
            sl = ift.draw_samples(pos, H, mini, 4, True)
            ift.random.pop_sseq()
        finally:
            config.set_cg_precision("fp64")
        out[prec] = _kl_checks(ift, sl, H, 8)
    from nifty_amd.minimization import geovi_batch
    p64 = [out["fp64"].samples.local_item(i) for i in range(8)]
    p32 = [out["fp32"].samples.local_item(i) for i in range(8)]
    for i, (a, b) in enumerate(zip(p32, p64)):
        va = torch.cat([a[k].val.reshape(-1) for k in a.keys()])
        vb = torch.cat([b[k].val.reshape(-1) for k in b.keys()])
        err = float(torch.linalg.vector_norm(va - vb) / torch.linalg.vector_norm(vb))
        assert err < 1e-4, (i, err)
    # the KL value (2.9e8, dominated by the data misfit at noise 0.01) moves
    # with the samples: its fp32 - fp64 change equals the first-order
    # prediction mean_i grad H(s_i) . (s32_i - s64_i) up to 5 % + 1e-9 KL
    v64, g64 = geovi_batch.kl_batch(H, p64)
    v32, _ = geovi_batch.kl_batch(H, p32)
    pred = np.mean([sum(float(torch.sum(g[k].val * (a[k].val - b[k].val))) for k in g.keys())
                    for g, a, b in zip(g64, p32, p64)])
    d = float(np.mean(v32) - np.mean(v64))
    assert abs(d - pred) <= 0.05 * abs(pred) + 1e-9 * abs(np.mean(v64)), (d, pred)
    assert abs(out["fp32"].value - float(np.mean(v32))) <= 1e-12 * abs(out["fp32"].value)


def test_c5_fp32_lazy_iterate_bitwise(ift, monkeypatch):
    """C5's fp32 storage with the deferred iterate of count-only chunks (fp32
    ring slots, the flush's fp32 x - alpha d): bitwise the per-step update"""
    from nifty_amd import _native, config
    from nifty_amd.minimization import fused_cg
    cf, lh, pos = _gauss_problem(ift, (256, 256))
    met, _ = _metric(ift, lh, pos)
    flushes = []
    orig = _native.cg_lazy_flush

    def spy(*a, **kw):
        flushes.append(a[6])
        return orig(*a, **kw)
    monkeypatch.setattr(_native, "cg_lazy_flush", spy)
    with ift.random.Context(6):
        es = [ift.QuadraticEnergy(0 * ift.from_random(cf.domain, "normal"), met, ift.from_random(cf.domain, "normal"))
              for _ in range(2)]
    out = {}
    config.set_cg_precision("fp32")
    try:
        core, W, shift = fused_cg.fusable_metric(met)
        for on in (True, False):
            monkeypatch.setattr(fused_cg, "LAZY", on)
            flushes.clear()
            cg = fused_cg.FusedCGBatch(core, W, shift, [ift.GradientNormController(iteration_limit=m) for m in (12, 27)])
            out[on] = cg.run(es)
            assert cg.path == "carry+chunk", cg.path
            assert bool(flushes) == on
    finally:
        config.set_cg_precision("fp64")
    for (e1, s1), (e2, s2) in zip(out[True], out[False]):
        assert s1 == s2
        for k in cf.domain.keys():
            assert torch.equal(e1.position[k].val, e2.position[k].val), k
