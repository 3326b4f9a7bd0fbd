"""Lock-step (batched) geoVI refinement vs the per-sample path.

draw_samples refines its local samples with NewtonCG; the batched driver
(minimization/geovi_batch.py) runs the same minimizer logic per sample with
batched evaluations.  Both must take the same decisions (inner-CG iteration counts, line-search
trial steps) and give the same samples within 10x the per-sample path's own
rounding sensitivity, for the bench's likelihood chain (sigmoid,
LOSResponse, Gaussian), a GeometryRemover Gaussian and a Poisson chain
(2 sqrt o exp)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CF_ARGS = dict(offset_mean=0, offset_std=(1e-3, 1e-6), fluctuations=(1., 0.8),
               loglogavgslope=(-3., 1), flexibility=(2, 1.), asperity=(0.5, 0.4))


@pytest.fixture(scope="module")
def ift(dev):
    import nifty_amd
    return nifty_amd


def _problem(ift, kind, n=64):
    sp = ift.RGSpace((n, n))
    cf = ift.SimpleCorrelatedField(sp, **CF_ARGS)
    ift.random.push_sseq_from_seed(11)
    if kind == "los":
        rng = ift.random.current_rng()
        nlos = 300
        starts = list(rng.random((nlos, 2)).T)
        ends = list(rng.random((nlos, 2)).T)
        R = ift.LOSResponse(sp, starts=starts, ends=ends)
        sig = R @ ift.sigmoid(cf)
        N = ift.ScalingOperator(R.target, 1e-3, np.float64)
        mock = ift.from_random(sig.domain, "normal")
        data = sig(mock) + N.draw_sample()
        lh = ift.GaussianEnergy(data, inverse_covariance=N.inverse) @ sig
    elif kind == "gauss":
        R = ift.GeometryRemover(sp)
        sig = R @ cf
        N = ift.ScalingOperator(R.target, 0.01, np.float64)
        mock = ift.from_random(sig.domain, "normal")
        data = sig(mock) + N.draw_sample()
        lh = ift.GaussianEnergy(data, inverse_covariance=N.inverse) @ sig
    else:
        sig = cf.exp()
        mock = ift.from_random(sig.domain, "normal")
        lam = sig(mock).val.cpu().numpy()
        counts = ift.random.current_rng().poisson(lam).astype(np.int64)
        lh = ift.PoissonianEnergy(ift.makeField(sp, counts)) @ sig
    pos = 0.1 * ift.from_random(cf.domain, "normal")
    ift.random.pop_sseq()
    return cf, lh, pos


def _draw(ift, cf, H, pos, newton, cg, batched):
    """one geoVI draw (2 mirrored pairs) with the decision trace on:
    (flat residual samples, trace events)"""
    from nifty_amd.minimization import geovi_batch, trace
    geovi_batch.ENABLED = batched
    trace.TRACE = []
    try:
        mini = ift.NewtonCG(ift.GradientNormController(iteration_limit=newton), max_cg_iterations=cg)
        ift.random.push_sseq_from_seed(5)
        sl = ift.draw_samples(pos, H, mini, 2, True)
        ift.random.pop_sseq()
        ev = trace.TRACE
    finally:
        trace.TRACE = None
        geovi_batch.ENABLED = True
    assert list(sl._n) == [False] * 4
    res = [np.concatenate([np.ravel(r[k].val.cpu().numpy()) for k in cf.domain.keys()]) for r in sl._r]
    return res, ev


# (Newton iterations, CG iterations per direction).  The batched and the
# per-sample path run the same decisions per sample; their floating-point
# paths differ (batched vs per-sample kernels, reduction layout).  The
# per-sample path is also run with the expansion point's xi moved by
# +-1e-15 (relative): the batched path's decision trace is held to the
# per-sample path's as tests/test_geovi_trace_gpu.py holds the build to the
# reference (tests/trace_compare.py), and its samples to 10x the per-sample
# path's own sensitivity (floor 1e-8) where the traces are stable.
@pytest.mark.parametrize("kind", ["los", "gauss", "poisson"])
@pytest.mark.parametrize("newton,cg", [(2, 5), (3, 20)])
def test_batched_refinement_matches_per_sample(ift, kind, newton, cg):
    from trace_compare import compare, our_events
    cf, lh, pos = _problem(ift, kind)
    # linear solves run to convergence (100 steps at 64^2) so that the
    # perturbed runs isolate the refinement's own sensitivity
    H = ift.StandardHamiltonian(lh, ift.GradientNormController(iteration_limit=100))
    bat, ebat = _draw(ift, cf, H, pos, newton, cg, True)
    seq, eseq = _draw(ift, cf, H, pos, newton, cg, False)
    sens, epert = 0.0, []
    for f in (1 + 1e-15, 1 - 1e-15):
        pp = ift.MultiField.from_dict({k: (v * f if k == "xi" else v) for k, v in pos.items()})
        per, ep = _draw(ift, cf, H, pp, newton, cg, False)
        epert.append(ep)
        sens = max([sens] + [np.linalg.norm(a - b) / np.linalg.norm(b) for a, b in zip(per, seq)])
    all_stable = True
    for s in range(4):
        n, stable, worst, log = compare(our_events(ebat, s), our_events(eseq, s),
                                        [our_events(e, s) for e in epert])
        print(f"{kind} newton={newton} sample {s}: {n} events, stable={stable}, worst {worst:.3g}", *log)
        all_stable &= stable
    tol = max(1e-8, 10 * sens)
    for a, b in zip(bat, seq):
        assert np.all(np.isfinite(a))
        err = np.linalg.norm(a - b) / np.linalg.norm(b)
        if all_stable:
            assert err <= tol, (kind, err, sens)


def test_batched_path_is_taken(ift):
    from nifty_amd.minimization import geovi_batch
    cf, lh, pos = _problem(ift, "los")
    dtype, f_lh = lh.get_transformation()
    mini = ift.NewtonCG(ift.GradientNormController(iteration_limit=1))
    assert geovi_batch.plan(mini, f_lh, None, pos) is not None


@pytest.mark.parametrize("kind", ["los", "gauss", "poisson"])
def test_batched_kl_matches_per_sample(ift, kind):
    """SampledKLEnergyClass value / gradient through geovi_batch.kl_batch vs
    the per-sample Hamiltonian evaluations (rtol 1e-12)."""
    from nifty_amd.minimization import geovi_batch
    cf, lh, pos = _problem(ift, kind)
    H = ift.StandardHamiltonian(lh, ift.GradientNormController(iteration_limit=5))
    ift.random.push_sseq_from_seed(7)
    sl = ift.draw_samples(pos, H, None, 2, True)
    ift.random.pop_sseq()
    dtype, _ = lh.get_transformation()
    assert geovi_batch.kl_batch(H, list(sl.local_iterator())) is not None
    kls = {}
    for enabled in (True, False):
        geovi_batch.ENABLED = enabled
        try:
            kls[enabled] = ift.SampledKLEnergyClass(sl, H, [], None, True)
        finally:
            geovi_batch.ENABLED = True
    a, b = kls[True], kls[False]
    assert abs(a.value - b.value) <= 1e-12 * abs(b.value)
    for k in cf.domain.keys():
        ga, gb = a.gradient[k].val.cpu().numpy(), b.gradient[k].val.cpu().numpy()
        assert np.linalg.norm(ga - gb) <= 1e-11 * max(np.linalg.norm(gb), 1e-300), k


@pytest.mark.parametrize("dtype", ["float64", "float32"])
def test_sigmoid_pair_bitwise(ift, dtype):
    """nft_sigmoid_pair (the batched geoVI pipeline's sigmoid stage) is
    bitwise the torch elementwise passes of pointwise._sigmoid, special
    values included."""
    import torch
    from nifty_amd import _native
    from nifty_amd.pointwise import _sigmoid
    dt = getattr(torch, dtype)
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    x = torch.cat([torch.randn(100003, dtype=torch.float64, device="cuda", generator=g) * 4,
                   torch.tensor([0.0, -0.0, 1e-300, -1e-300, 20.0, -20.0, 400.0, -400.0, float("inf"),
                                 float("-inf")], dtype=torch.float64, device="cuda")]).to(dt)
    v0, d0 = _sigmoid(x)
    v1, d1 = _native.sigmoid_pair(x, torch.empty_like(x), torch.empty_like(x))
    assert torch.equal(v0, v1) and torch.equal(d0, d1)
    assert torch.equal(torch.signbit(v0), torch.signbit(v1)) and torch.equal(torch.signbit(d0), torch.signbit(d1))
