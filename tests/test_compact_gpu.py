"""Compaction of the lock-step batched CG (fused_cg.FusedCGBatch.run_packed):
once some right-hand sides stop, the live ones continue in smaller buffers
(and, for per-sample Newton metrics, a metric restricted to them).  Per RHS
the arithmetic does not depend on the batch size, so every result is
bitwise that of the uncompacted batch and of sequential solves."""
import copy

import numpy as np
import pytest
import torch

from test_geovi_batch_gpu import CF_ARGS, _problem  # noqa: F401
from test_parity_gpu import _gaussian, _los_problem, golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ift(dev):
    import nifty_amd
    return nifty_amd


def _metric(ift, which):
    from nifty_amd.minimization.fused_cg import fusable_metric
    if which == "los":
        cf, lh, pos = _los_problem(ift, golden("losmetric64.npz"))
    else:
        cf, lh, pos = _gaussian(ift, golden("metric128.npz"))
    dtype, f_lh = lh.get_transformation()
    fl = f_lh(ift.Linearization.make_var(pos))
    A = (ift.SandwichOperator.make(fl.jac, ift.ScalingOperator(f_lh.target, 1., dtype))
         + ift.ScalingOperator(fl.domain, 1., float))
    return cf, A, fusable_metric(A)


def _energies(ift, cf, A, k, seed):
    with ift.random.Context(seed):
        return [ift.QuadraticEnergy(0.1 * ift.from_random(cf.domain, "normal"), A,
                                    ift.from_random(cf.domain, "normal")) for _ in range(k)]


@pytest.mark.parametrize("which", ["los", "gauss"])
def test_compacted_count_only_vs_sequential(ift, which):
    """count-only controllers with different limits (queued chunks, then
    compaction; 25 crosses the nreset=20 residual refresh): bitwise the
    sequential single solves"""
    from nifty_amd.minimization.fused_cg import FusedCG, FusedCGBatch
    cf, A, (core, W, shift) = _metric(ift, which)
    es = _energies(ift, cf, A, 3, 3)
    lims = [4, 11, 25]
    seq = [FusedCG(core, W, shift, ift.GradientNormController(iteration_limit=m)).run(e) for e, m in zip(es, lims)]
    from nifty_amd.minimization import fused_cg
    cg = FusedCGBatch(core, W, shift, [ift.GradientNormController(iteration_limit=m) for m in lims])
    n0 = fused_cg.STATS["carry_iters"]
    bat = cg.run(es)
    assert cg.compactions >= 1
    # the carried iteration (amplitude keys in the two-phase kernels; the
    # Gaussian's pointwise W in the forward transform's epilogue) ran before
    # and after the compaction
    assert cg.path == "carry+chunk", cg.path
    assert fused_cg.STATS["carry_iters"] - n0 >= 20
    for (e1, s1), (e2, s2) in zip(seq, bat):
        assert s1 == s2
        for key in cf.domain.keys():
            assert torch.equal(e1.position[key].val, e2.position[key].val), key


@pytest.mark.parametrize("which", ["los", "gauss"])
def test_compacted_value_controllers_bitwise(ift, which, monkeypatch):
    """value-driven controllers stopping at different iterations: compacted
    and uncompacted batches agree bitwise, with the same checks"""
    from nifty_amd.minimization import fused_cg
    cf, A, (core, W, shift) = _metric(ift, which)
    es = _energies(ift, cf, A, 4, 8)
    ctls = [ift.AbsDeltaEnergyController(d, iteration_limit=m)
            for d, m in ((1e-1, 40), (1e-3, 7), (1e-6, 16), (1e-9, 30))]
    out = {}
    for on in (False, True):
        monkeypatch.setattr(fused_cg, "COMPACT", on)
        cs = [copy.deepcopy(c) for c in ctls]
        cg = fused_cg.FusedCGBatch(core, W, shift, cs)
        out[on] = (cg.run(es), [c._itcount for c in cs], cg.compactions)
    assert out[True][2] >= 1 and out[False][2] == 0
    assert out[True][1] == out[False][1]
    assert len(set(out[True][1])) > 1
    for (e1, s1), (e2, s2) in zip(out[False][0], out[True][0]):
        assert s1 == s2
        for key in cf.domain.keys():
            assert torch.equal(e1.position[key].val, e2.position[key].val), key


def test_compacted_newton_directions_bitwise(ift, monkeypatch):
    """batched geoVI refinement with the demo's value-driven Newton
    controllers: the NewtonCG direction solves (per-sample metrics, restricted
    by core.subset on compaction) give bitwise the uncompacted samples"""
    from nifty_amd.minimization import fused_cg
    cf, lh, pos = _problem(ift, "los")
    H = ift.StandardHamiltonian(lh, ift.AbsDeltaEnergyController(deltaE=0.05, iteration_limit=30))
    res, ncomp = {}, {}
    orig = fused_cg.FusedCGBatch.run_packed

    def counting(self, *a):
        r = orig(self, *a)
        ncomp[on] = ncomp.get(on, 0) + self.compactions
        return r
    monkeypatch.setattr(fused_cg.FusedCGBatch, "run_packed", counting)
    for on in (False, True):
        monkeypatch.setattr(fused_cg, "COMPACT", on)
        mini = ift.NewtonCG(ift.AbsDeltaEnergyController(deltaE=0.5, convergence_level=2, iteration_limit=4))
        ift.random.push_sseq_from_seed(21)
        sl = ift.draw_samples(pos, H, mini, 2, True)
        ift.random.pop_sseq()
        res[on] = [np.concatenate([np.ravel(r[k].val.cpu().numpy()) for k in cf.domain.keys()]) for r in sl._r]
    assert ncomp.get(True, 0) >= 1 and ncomp.get(False, 0) == 0
    for a, b in zip(res[False], res[True]):
        assert np.array_equal(a, b)


def test_fold_in_los_adjoint_bitwise(ift, monkeypatch):
    """the carried iteration's curvature fold inside the LOS adjoint launch
    (nft_los_adjoint_fold) gives bitwise the separate nft_fold_partials"""
    from nifty_amd import _native
    from nifty_amd.minimization.fused_cg import FusedCGBatch
    cf, A, (core, W, shift) = _metric(ift, "los")
    assert getattr(W, "supports_fold", False)
    es = _energies(ift, cf, A, 3, 5)
    lims = [6, 9, 23]
    calls = []
    orig = _native.los_adjoint_batched

    def spy(*a, **kw):
        calls.append(kw.get("fold") is not None)
        return orig(*a, **kw)
    monkeypatch.setattr(_native, "los_adjoint_batched", spy)
    out = {}
    for on in (True, False):
        monkeypatch.setattr(W, "supports_fold", on)
        calls.clear()
        cg = FusedCGBatch(core, W, shift, [ift.GradientNormController(iteration_limit=m) for m in lims])
        out[on] = cg.run(es)
        assert cg.path.startswith("carry"), cg.path
        assert any(calls) == on
    for (e1, s1), (e2, s2) in zip(out[True], out[False]):
        assert s1 == s2
        for key in cf.domain.keys():
            assert torch.equal(e1.position[key].val, e2.position[key].val), key


@pytest.mark.parametrize("which", ["los", "gauss"])
def test_lazy_iterate_bitwise(ift, which, monkeypatch):
    """the deferred iterate of count-only chunks (directions in ring slots, x
    brought up to date once per chunk, nft_cg_lazy_flush) gives bitwise the
    per-step update -- across the residual refreshes and a compaction"""
    from nifty_amd import _native
    from nifty_amd.minimization import fused_cg
    # these small 2-D grids take the fused prologue + R2C pass, which keeps
    # its direction in place: the row-staged prologue here
    monkeypatch.setenv("NFT_PRO_R2C", "0")
    cf, A, (core, W, shift) = _metric(ift, which)
    es = _energies(ift, cf, A, 4, 9)
    lims = [7, 13, 30, 45]
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
        cg = fused_cg.FusedCGBatch(core, W, shift, [ift.GradientNormController(iteration_limit=m) for m in lims])
        out[on] = cg.run(es)
        assert cg.path == "carry+chunk", cg.path
        assert bool(flushes) == on
        if on:
            assert cg.compactions >= 1 and sum(flushes) >= 30
    for (e1, s1), (e2, s2) in zip(out[True], out[False]):
        assert s1 == s2
        for key in cf.domain.keys():
            assert torch.equal(e1.position[key].val, e2.position[key].val), key


def test_fold_in_adjoint_r2c_bitwise(ift, monkeypatch):
    """the carried iteration's curvature fold inside the adjoint transform's
    R2C row pass (nft_hartley_fuse.fold_*, pointwise W) gives bitwise the
    separate nft_fold_partials"""
    from nifty_amd import _native
    from nifty_amd.library import correlated_fields_simple as cfs
    from nifty_amd.minimization.fused_cg import FusedCGBatch
    cf, A, (core, W, shift) = _metric(ift, "gauss")
    assert torch.is_tensor(W)
    es = _energies(ift, cf, A, 3, 5)
    lims = [6, 9, 23]
    calls = []
    orig = _native.hartley_fused

    def spy(*a, **kw):
        calls.append(kw.get("fold") is not None)
        return orig(*a, **kw)
    monkeypatch.setattr(_native, "hartley_fused", spy)
    out = {}
    for on in (True, False):
        monkeypatch.setattr(cfs, "_FOLD_R2C", on)
        calls.clear()
        cg = FusedCGBatch(core, W, shift, [ift.GradientNormController(iteration_limit=m) for m in lims])
        out[on] = cg.run(es)
        assert cg.path.startswith("carry"), cg.path
        assert any(calls) == on
    for (e1, s1), (e2, s2) in zip(out[True], out[False]):
        assert s1 == s2
        for key in cf.domain.keys():
            assert torch.equal(e1.position[key].val, e2.position[key].val), key


@pytest.mark.parametrize("shape", [(16, 256), (8, 2048), (8, 4096), (4, 8192), (8, 16, 64), (4, 96)])
def test_hartley_carried_fold_direct(shape):
    """nft_hartley_fuse.fold_*: the sums bitwise nft_fold_partials' for every
    R2C workgroup size (256 / 512 / 1024 threads), the transform unchanged; a
    geometry without the engine-v2 R2C pass (4 x 96) folds in its own launch"""
    from nifty_amd import _native
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(11)
    x = torch.randn(shape, generator=g, dtype=torch.float64).to(dev)
    axes = tuple(range(len(shape)))
    nrhs, nb = 3, 2311
    part = torch.randn((nrhs, nb), generator=g, dtype=torch.float64).to(dev)
    ref = torch.full((nrhs, 5), -1.0, dtype=torch.float64, device=dev)
    _native._check(_native.load().nft_fold_partials(_native.ptr(part), nb, nrhs, _native.ptr(ref), 5,
                                                    _native.stream_ptr()))
    got = torch.full((nrhs, 5), -1.0, dtype=torch.float64, device=dev)
    h0 = torch.empty_like(x)
    h1 = torch.empty_like(x)
    _native.hartley_fused(h0, axes, 1.0, x=x)
    _native.hartley_fused(h1, axes, 1.0, x=x, fold=(part, nb, nrhs, got.data_ptr(), 5))
    torch.cuda.synchronize()
    assert torch.equal(h0, h1)
    assert torch.equal(got, ref)
    assert torch.equal(got[:, 1:], torch.full_like(got[:, 1:], -1.0))
