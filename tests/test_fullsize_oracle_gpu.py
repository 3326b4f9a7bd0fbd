"""BASELINE.json configs at their FULL sizes against the CPU oracle (oracle/,
the numpy / scipy restatement pinned to the reference's golden vectors in
tests/test_oracle.py), on the bench's own problems (bench.build_problem: seed
27 mock data, expansion point 0.1 N(0,1)):

  C3  2048^2 CF, sigmoid, LOSResponse(16384), Gaussian 1e-3   (the bench workload)
  C2  1024^2 CF, exp, Poisson counts
  C5  4096^2 CF, Gaussian 0.01 (fp64 storage)
  C4  512^3  CF (no asperity), Gaussian 0.01

One application of the geoVI / MGVI sampling metric M = 1 + J^T J of the
likelihood's whitened transformation (kl_energies.py:147-153 through
sandwich_operator.py:41-95) per config at rtol 1e-12 per latent key, and at C3
five iterations of the linear CG (conjugate_gradient.py:48-126, the bench's
count-only GradientNormController) at rtol 1e-9 on the iterate and the
energy.  The oracle runs numpy + scipy.fft on at most 16 host cores (the GPU
box's share); each case takes 5-60 s of host time."""
import os

import numpy as np
import pytest
import torch

import bench
from oracle.cf import CFOracle
from oracle.geovi import GaussWhitened, LOSWhitened, PoissonWhitened
from oracle.sampling import GradNormCtl, axpy, conjugate_gradient

pytestmark = pytest.mark.gpu

WORKERS = max(1, min(16, os.cpu_count() or 1))


@pytest.fixture(scope="module")
def ift(dev):
    import nifty_amd
    return nifty_amd


def _setup(ift, config):
    cfg = bench.CONFIGS[config]
    n = cfg["shape"][0]
    cf, R, lh, pos, _ = bench.build_problem(ift, n, 16384, config)
    dtype, f_lh = lh.get_transformation()
    fl = f_lh(ift.Linearization.make_var(pos))
    met = (ift.SandwichOperator.make(fl.jac, ift.ScalingOperator(f_lh.target, 1., dtype))
           + ift.ScalingOperator(fl.domain, 1., float))
    shape = tuple(cf.target.shape)
    o = CFOracle(shape, **(dict(bench.CF_ARGS, asperity=None) if len(shape) == 3 else bench.CF_ARGS))
    if cfg["lik"] == "los":
        rows, cols, w = R.coo
        olh = LOSWhitened(o, rows, cols, w, R.target.shape[0], 1e-3)
    elif cfg["lik"] == "poisson":
        olh = PoissonWhitened(o)
    else:
        olh = GaussWhitened(o, 0.01)
    lat = {k: pos[k].val.cpu().numpy() for k in cf.domain.keys()}
    return cf, met, olh, lat


def _rel(a, b):
    return float(np.linalg.norm(np.ravel(a - b)) / max(np.linalg.norm(np.ravel(b)), 1e-300))


@pytest.mark.parametrize("config", ["C3", "C2", "C5", "C4"])
def test_sampling_metric_full_size_vs_oracle(ift, config):
    import scipy.fft
    cf, met, olh, lat = _setup(ift, config)
    with ift.random.Context(101):
        v = ift.from_random(cf.domain, "normal")
    got = met(v)
    vn = {k: v[k].val.cpu().numpy() for k in cf.domain.keys()}
    with scipy.fft.set_workers(WORKERS):
        ref = axpy(1., vn, olh.vjp(lat, olh.jvp(lat, vn)))
    for k in cf.domain.keys():
        err = _rel(got[k].val.cpu().numpy(), np.reshape(ref[k], np.shape(vn[k])))
        assert err < 1e-12, (config, k, err)


def test_cg_five_steps_c3_vs_oracle(ift):
    """the bench's linear CG (count-only controller, the carried batched
    iteration) five steps from x0 = 0 on b ~ N(0, 1) at 2048^2 with the LOS
    response: iterate and energy against the oracle's CG at rtol 1e-9"""
    import scipy.fft
    cf, met, olh, lat = _setup(ift, "C3")
    with ift.random.Context(202):
        b = ift.from_random(cf.domain, "normal")
    ic = ift.GradientNormController(iteration_limit=5)
    en, st = ift.ConjugateGradient(ic)(ift.QuadraticEnergy(0 * b, met, b))
    assert st == ic.CONVERGED
    bn = {k: b[k].val.cpu().numpy() for k in cf.domain.keys()}
    zero = {k: np.zeros_like(x) for k, x in bn.items()}

    def M(x):
        return axpy(1., x, {k: np.reshape(y, np.shape(x[k])) for k, y in olh.vjp(lat, olh.jvp(lat, x)).items()})
    with scipy.fft.set_workers(WORKERS):
        xo, sto, it = conjugate_gradient(M, zero, bn, GradNormCtl(iteration_limit=5))
        Ax = M(xo)
    assert sto == 0 and it == 5
    for k in cf.domain.keys():
        err = _rel(en.position[k].val.cpu().numpy(), xo[k])
        assert err < 1e-9, (k, err)
    val = 0.5 * sum(float(np.vdot(xo[k], Ax[k])) for k in xo) - sum(float(np.vdot(bn[k], xo[k])) for k in xo)
    assert abs(en.value - val) <= 1e-9 * abs(val), (en.value, val)
