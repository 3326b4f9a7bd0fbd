"""The carried CG iteration for pointwise likelihood weights (Gaussian with
GeometryRemover, Poisson): the data-space curvature (J d).W(J d) formed by the
forward transform's epilogue (nft_hartley_fuse.quad_*), the update carried by
the adjoint's epilogue and the two-phase amplitude kernels -- against the
separate direction / curvature / update passes on the same metric
(src/minimization/conjugate_gradient.py:84-124; energy_operators.py:578-579,
624-625).  The two differ only in how curv = d.(A d) is rounded, so the
iterates agree to rtol 1e-9 after 10 steps (count-only controllers, whose
decisions cannot change)."""
import numpy as np
import pytest
import torch

from test_parity_gpu import CF_ARGS, _gaussian, golden, mf

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ift(dev):
    import nifty_amd
    return nifty_amd


def _poisson(ift):
    G = golden("poisson64.npz")
    sp = ift.RGSpace((64, 64))
    cf = ift.SimpleCorrelatedField(sp, **CF_ARGS)
    lh = ift.PoissonianEnergy(ift.makeField(sp, G["counts"])) @ cf.exp()
    return cf, lh, mf(ift, cf.domain, G, "pos_")


def _metric(ift, which):
    from nifty_amd.minimization.fused_cg import fusable_metric
    cf, lh, pos = _poisson(ift) if which == "poisson" else _gaussian(ift, golden("metric128.npz"))
    dtype, f_lh = lh.get_transformation()
    fl = f_lh(ift.Linearization.make_var(pos))
    A = (ift.SandwichOperator.make(fl.jac, ift.ScalingOperator(f_lh.target, 1., dtype))
         + ift.ScalingOperator(fl.domain, 1., float))
    return cf, A, fusable_metric(A)


@pytest.mark.parametrize("which", ["gauss", "poisson"])
def test_pointwise_carried_vs_separate(ift, which, monkeypatch):
    from nifty_amd.minimization import fused_cg
    cf, A, (core, W, shift) = _metric(ift, which)
    assert torch.is_tensor(W) and core.pointwise_quad_blocks(W) > 0
    with ift.random.Context(5):
        es = [ift.QuadraticEnergy(0.1 * ift.from_random(cf.domain, "normal"), A,
                                  ift.from_random(cf.domain, "normal")) for _ in range(4)]
    out = {}
    for carry in (True, False):
        monkeypatch.setattr(fused_cg, "CURV_DATA", carry)
        n0 = fused_cg.STATS["carry_iters"]
        cg = fused_cg.FusedCGBatch(core, W, shift, [ift.GradientNormController(iteration_limit=10)
                                                    for _ in range(4)])
        out[carry] = cg.run(es)
        if carry:
            assert cg.path == "carry+chunk", cg.path
            assert fused_cg.STATS["carry_iters"] - n0 >= 5
        else:
            assert cg.path.startswith("plain"), cg.path
    for (e1, s1), (e2, s2) in zip(out[True], out[False]):
        assert s1 == s2
        for k in cf.domain.keys():
            a, b = e1.position[k].val, e2.position[k].val
            err = float(torch.linalg.vector_norm(a - b) / torch.linalg.vector_norm(b))
            assert err < 1e-9, (k, err)


def test_pointwise_quad_partials(ift):
    """the forward transform's quadratic-form partials sum to (J d).W(J d)
    computed from the stored s = W J d (rtol 1e-13), for every RHS of a
    batch; s itself equals W times the plain forward transform bitwise"""
    from nifty_amd import _native
    cf, A, (core, W, shift) = _metric(ift, "gauss")
    k = 3
    lay = core.layout
    n = lay.size
    D = torch.randn((k, n), dtype=torch.float64, device=W.device)
    nq = core.pointwise_quad_blocks(W)
    da = core.mv_amp_jvp(D)
    qpart = torch.full((k, nq + 5), np.nan, dtype=torch.float64, device=W.device)
    Q = torch.zeros_like(D)
    core.mv_grid(D, da, Q, W, 0.0, qpart=qpart[:, :nq])
    s = core._mv_bufs(k)["s"].clone()
    Q2 = torch.zeros_like(D)
    da = core.mv_amp_jvp(D)
    core.mv_grid(D, da, Q2, W, 0.0)
    # the plain path forms s * W in torch from the unweighted transform: the
    # stored product is the same rounding
    assert torch.equal(Q, Q2)
    for b in range(k):
        h = s[b] / W
        ref = float(torch.sum(h * s[b]))
        got = float(torch.sum(qpart[b, :nq]))
        assert abs(got - ref) <= 1e-13 * abs(ref), (b, got, ref)
    assert bool(torch.all(torch.isnan(qpart[:, nq:])))


@pytest.mark.parametrize("which", ["gauss", "los"])
def test_fp32_carried_vs_fp64(ift, which):
    """fp32 storage (config.set_cg_precision("fp32")): the carried iteration
    runs (two-phase amplitude kernels and transforms on fp32 operands, fp64
    partials and scalars) and stays within rtol 1e-4 of the fp64 solve
    (BASELINE.json C5)."""
    from nifty_amd import config
    from nifty_amd.minimization import fused_cg
    if which == "los":
        from test_compact_gpu import _metric as _los_metric
        cf, A, (core, W, shift) = _los_metric(ift, "los")
    else:
        cf, A, (core, W, shift) = _metric(ift, which)
    with ift.random.Context(6):
        es = [ift.QuadraticEnergy(0 * ift.from_random(cf.domain, "normal"), A,
                                  ift.from_random(cf.domain, "normal")) for _ in range(4)]
    out = {}
    for prec in ("fp64", "fp32"):
        config.set_cg_precision(prec)
        try:
            n0 = fused_cg.STATS["carry_iters"]
            cg = fused_cg.FusedCGBatch(core, W, shift, [ift.GradientNormController(iteration_limit=8)
                                                        for _ in range(4)])
            out[prec] = cg.run(es)
            assert cg.path == "carry+chunk", (prec, cg.path)
            assert fused_cg.STATS["carry_iters"] - n0 >= 4
        finally:
            config.set_cg_precision("fp64")
    for (e1, s1), (e2, s2) in zip(out["fp32"], out["fp64"]):
        assert s1 == s2
        for k in cf.domain.keys():
            a, b = e1.position[k].val, e2.position[k].val
            err = float(torch.linalg.vector_norm(a - b) / torch.linalg.vector_norm(b))
            assert err < 1e-4, (k, err)
