"""The folded prologue fused with the forward transform's R2C row pass
(csrc/nft_pro_r2c.hip: by default the carried CG iteration's pass on 2-D
grids with rows of 512 or 1024, forced here with NFT_PRO_R2C=2 for longer
rows too) against the split passes (pro_rows_kernel + the
persistent R2C pass, NFT_PRO_R2C=0) on the same sampling metric
(src/minimization/conjugate_gradient.py:84-124 over
src/library/correlated_fields_simple.py:86-127).  The fused pass packs the
mirror rows g, n0 - g into one complex FFT where the R2C pass packs rows
2l, 2l + 1, so the half spectra differ in the last bits: the iterates agree to
rtol 1e-8 after 10 steps (count-only controllers, whose decisions cannot
change; ten steps amplify the last-bit differences to ~1e-9 on some keys); per right-hand side the fused pass does not depend on the batch
(single == batched, bitwise)."""
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


def _problem(ift, shape, kind):
    sp = ift.RGSpace(shape)
    cf = ift.SimpleCorrelatedField(sp, **CF_ARGS)
    ift.random.push_sseq_from_seed(31)
    if kind == "los":
        rng = ift.random.current_rng()
        nlos = 2000
        R = ift.LOSResponse(sp, starts=list(rng.random((nlos, 2)).T), ends=list(rng.random((nlos, 2)).T))
        sr = R @ ift.sigmoid(cf)
        N = ift.ScalingOperator(R.target, 1e-3, np.float64)
        data = sr(ift.from_random(cf.domain, "normal")) + N.draw_sample()
        lh = ift.GaussianEnergy(data, inverse_covariance=N.inverse) @ sr
    else:
        R = ift.GeometryRemover(sp)
        N = ift.ScalingOperator(R.target, 0.01, np.float64)
        data = R(cf(ift.from_random(cf.domain, "normal"))) + N.draw_sample()
        lh = ift.GaussianEnergy(data, inverse_covariance=N.inverse) @ (R @ cf)
    pos = 0.1 * ift.from_random(cf.domain, "normal")
    ift.random.pop_sseq()
    dtype, f_lh = lh.get_transformation()
    fl = f_lh(ift.Linearization.make_var(pos))
    A = (ift.SandwichOperator.make(fl.jac, ift.ScalingOperator(f_lh.target, 1., dtype))
         + ift.ScalingOperator(fl.domain, 1., float))
    return cf, A


def _energies(ift, cf, A, k, seed=5):
    with ift.random.Context(seed):
        return [ift.QuadraticEnergy(0.1 * ift.from_random(cf.domain, "normal"), A,
                                    ift.from_random(cf.domain, "normal")) for _ in range(k)]


def _run(ift, cf, A, es, iters, fused, monkeypatch):
    from nifty_amd.minimization import fused_cg
    from nifty_amd.minimization.fused_cg import fusable_metric
    monkeypatch.setenv("NFT_PRO_R2C", "2" if fused else "0")
    core, W, shift = fusable_metric(A)
    cg = fused_cg.FusedCGBatch(core, W, shift, [ift.GradientNormController(iteration_limit=iters) for _ in es])
    out = cg.run(es)
    assert cg.path == "carry+chunk", cg.path
    return out


def _rel(a, b):
    return float(torch.linalg.vector_norm(a - b) / torch.linalg.vector_norm(b))


@pytest.mark.parametrize("shape,kind", [((512, 512), "los"), ((256, 1024), "gauss"), ((1024, 512), "gauss"),
                                        ((256, 2048), "gauss")])
def test_pro_r2c_vs_split(ift, shape, kind, monkeypatch):
    cf, A = _problem(ift, shape, kind)
    es = _energies(ift, cf, A, 4)
    res = {f: _run(ift, cf, A, es, 10, f, monkeypatch) for f in (True, False)}
    for (e1, s1), (e2, s2) in zip(res[True], res[False]):
        assert s1 == s2
        for k in cf.domain.keys():
            err = _rel(e1.position[k].val, e2.position[k].val)
            assert err < 1e-8, (k, err)
        assert abs(e1.value - e2.value) <= 1e-9 * abs(e2.value)


def test_pro_r2c_launched_and_batch_independent(ift, monkeypatch):
    from nifty_amd import _native
    cf, A = _problem(ift, (512, 512), "los")
    es = _energies(ift, cf, A, 3)
    with _native.LaunchProfile() as p:
        _run(ift, cf, A, es[:1], 2, True, monkeypatch)
    labels = {lab for lab, _ in p.records}
    assert "pro_r2c+dir" in labels, sorted(labels)
    assert "pro_fold+dir" not in labels
    one = _run(ift, cf, A, es[:1], 12, True, monkeypatch)
    three = _run(ift, cf, A, es, 12, True, monkeypatch)
    for k in cf.domain.keys():
        assert torch.equal(one[0][0].position[k].val, three[0][0].position[k].val), k


def test_pro_r2c_fp32(ift, monkeypatch):
    """C5's fp32 storage through the fused pass: the whole latent vector
    within rtol 1e-4 of the fp64 solve (BASELINE.json C5; single scalar keys
    move by up to ~2e-4 relative after 8 steps at 512^2)"""
    from nifty_amd import config
    cf, A = _problem(ift, (512, 512), "gauss")
    es = _energies(ift, cf, A, 2)
    r64 = _run(ift, cf, A, es, 8, True, monkeypatch)
    config.set_cg_precision("fp32")
    try:
        r32 = _run(ift, cf, A, es, 8, True, monkeypatch)
    finally:
        config.set_cg_precision("fp64")
    for (e1, _), (e2, _) in zip(r32, r64):
        a = torch.cat([e1.position[k].val.reshape(-1) for k in cf.domain.keys()])
        b = torch.cat([e2.position[k].val.reshape(-1) for k in cf.domain.keys()])
        assert _rel(a, b) < 1e-4


@pytest.mark.parametrize("shape,kind", [((512, 512), "los"), ((256, 1024), "gauss")])
def test_pro_r2c_lazy_iterate_bitwise(ift, shape, kind, monkeypatch):
    """the fused pass with the deferred iterate of count-only chunks (its
    directions in ring slots, nft_cg_lazy_flush) gives bitwise the per-step
    update, across the residual refreshes and a compaction"""
    from nifty_amd import _native
    from nifty_amd.minimization import fused_cg
    cf, A = _problem(ift, shape, kind)
    es = _energies(ift, cf, A, 3)
    flushes = []
    orig = _native.cg_lazy_flush

    def spy(*a, **kw):
        flushes.append(a[6])
        return orig(*a, **kw)
    monkeypatch.setattr(_native, "cg_lazy_flush", spy)
    out = {}
    for on in (True, False):
        monkeypatch.setattr(fused_cg, "LAZY", on)
        flushes.clear()
        monkeypatch.setenv("NFT_PRO_R2C", "2")
        from nifty_amd.minimization.fused_cg import fusable_metric
        core, W, shift = fusable_metric(A)
        cg = fused_cg.FusedCGBatch(core, W, shift, [ift.GradientNormController(iteration_limit=m)
                                                    for m in (9, 24, 31)])
        out[on] = cg.run(es)
        assert cg.path == "carry+chunk", cg.path
        assert bool(flushes) == on
    for (e1, s1), (e2, s2) in zip(out[True], out[False]):
        assert s1 == s2
        for key in cf.domain.keys():
            assert torch.equal(e1.position[key].val, e2.position[key].val), key
