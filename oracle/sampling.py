"""Oracle: sampling-metric CG and MGVI sample drawing for a correlated field
under a pointwise likelihood (Gaussian with GeometryRemover response, or
Poisson with exp signal).  TEST INFRASTRUCTURE ONLY.

Restates
  ConjugateGradient.__call__          src/minimization/conjugate_gradient.py:48-126
  QuadraticEnergy                     src/minimization/quadratic_energy.py:31-39
  Gradient/AbsDelta controllers       src/minimization/iteration_controllers.py:148-221, 356-423
  SamplingEnabler.special_draw_sample src/operators/sampling_enabler.py:64-86
  draw_samples (MGVI branch)          src/minimization/kl_energies.py:90-158
on latent dicts {key: ndarray} in sorted-key order.
"""
import numpy as np

from .cf import CFOracle


def _keys(d):
    return sorted(d.keys())


def vdot(a, b):
    return float(sum(np.vdot(a[k], b[k]) for k in _keys(a)))


def axpy(alpha, x, y):
    return {k: y[k] + alpha * x[k] for k in _keys(y)}


class PointwiseLikelihood:
    """Whitened likelihood transformation  f = sqrt(w(s)) * s-response  of a
    correlated field; the sampling metric is 1 + J^T W J with W = w(s0)."""

    def __init__(self, cf, kind, data, noise_var=None):
        self.cf = cf
        self.kind = kind
        self.data = data
        self.noise_var = noise_var

    def weight(self, lat0):
        s0 = self.cf.value(lat0)
        if self.kind == "gaussian":
            return np.full(s0.shape, 1. / self.noise_var)
        if self.kind == "poisson":  # f = 2 sqrt(exp(s)): df/ds = exp(s/2)
            return np.exp(s0)
        raise ValueError(self.kind)


class LOSLikelihood:
    """Tomography likelihood of config C3: d = R sigmoid(s) + n, n ~ N(0, var)
    (getting_started_3.py): the sampling metric's middle is
    diag(sig') R^T N^-1 R diag(sig'), sig = 0.5 + 0.5 tanh (pointwise.py:148).
    R is given as COO arrays (rows, cols, float32 weights), applied with
    scipy.sparse as src/library/los_response.py:226-233 does."""

    def __init__(self, cf, rows, cols, wgt, nlos, noise_var):
        import scipy.sparse
        self.cf = cf
        self.R = scipy.sparse.coo_matrix((wgt, (rows, cols)), shape=(nlos, int(np.prod(cf.shape)))).tocsr()
        self.noise_var = noise_var

    def middle(self, lat0):
        s0 = self.cf.value(lat0)
        t = np.tanh(s0)
        dsig = 0.5 * (1. - t * t)
        R, iv = self.R, 1. / self.noise_var

        def apply(v):
            y = R @ (dsig * v).ravel()
            return dsig * (R.T @ (iv * y)).reshape(v.shape)
        return apply


class SamplingMetric:
    """x -> x + J^T W J x; W is a pointwise weight array or a callable middle."""

    def __init__(self, cf, lat0, W):
        self.cf, self.lat0, self.W = cf, lat0, W

    def __call__(self, x):
        s = self.cf.jvp(self.lat0, x)
        s = self.W(s) if callable(self.W) else self.W * s
        g = self.cf.vjp(self.lat0, s)
        return {k: x[k] + np.reshape(g[k], np.shape(x[k])) for k in _keys(x)}


class GradNormCtl:
    def __init__(self, iteration_limit=None, tol_abs_gradnorm=None):
        self.lim, self.tol = iteration_limit, tol_abs_gradnorm

    def start(self, value, gnorm):
        self.it, self.cc = -1, 0
        return self.check(value, gnorm)

    def check(self, value, gnorm):
        self.it += 1
        if self.tol is not None and gnorm <= self.tol:
            self.cc += 1
        else:
            self.cc = max(0, self.cc - 1)
        if self.lim is not None and self.it >= self.lim:
            return 0
        return 0 if self.cc >= 1 else 1


class AbsDeltaCtl:
    def __init__(self, deltaE, convergence_level=1, iteration_limit=None):
        self.dE, self.cl, self.lim = deltaE, convergence_level, iteration_limit

    def start(self, value, gnorm):
        self.it, self.cc, self.Eold = -1, 0, 0.
        return self.check(value, gnorm)

    def check(self, value, gnorm):
        self.it += 1
        inc = self.it > 0 and abs(self.Eold - value) < self.dE
        self.Eold = value
        self.cc = self.cc + 1 if inc else max(0, self.cc - 1)
        if self.lim is not None and self.it >= self.lim:
            return 0
        return 0 if self.cc >= self.cl else 1


def quad_value(x, Ax, b):
    return 0.5 * vdot(x, Ax) - vdot(b, x)


def conjugate_gradient(A, x, b, ctl, grad=None, nreset=20, trace=None):
    """Returns (x, status, niter).  status: 0 converged, 2 error."""
    Ax = A(x) if grad is None else axpy(1., b, grad)
    r = axpy(-1., b, Ax) if grad is None else grad
    value = quad_value(x, Ax, b)
    if ctl.start(value, np.sqrt(max(vdot(r, r), 0.))) != 1:
        return x, 0, 0
    d = r
    gprev = vdot(r, d)
    if np.isnan(gprev):
        return x, 2, 0
    if gprev == 0:
        return x, 0, 0
    ii = 0
    niter = 0
    while True:
        q = A(d)
        curv = vdot(d, q)
        if np.isnan(curv) or curv == 0.:
            return x, 2, niter
        alpha = gprev / curv
        if alpha < 0:
            return x, 2, niter
        ii += 1
        niter += 1
        if ii < nreset:
            r = axpy(-alpha, q, r)
            x = axpy(-alpha, d, x)
            Ax = axpy(1., b, r)
        else:
            x = axpy(-alpha, d, x)
            Ax = A(x)
            r = axpy(-1., b, Ax)
            ii = 0
        gamma = vdot(r, r)
        if np.isnan(gamma) or gamma < 0:
            return x, 2, niter
        if gamma == 0:
            return x, 0, niter
        value = quad_value(x, Ax, b)
        if trace is not None:
            trace.append((curv, alpha, gamma, value))
        if ctl.check(value, np.sqrt(gamma)) != 1:
            return x, 0, niter
        d = axpy(max(0, gamma / gprev), d, r)
        gprev = gamma


def draw_mgvi(cf, lh, lat0, n_samples, mirror, seed_seq, ctl_factory, nreset=20):
    """MGVI residuals (kl_energies.py:131-149) for a pointwise likelihood;
    `seed_seq` is the parent SeedSequence (the reference's top of stack)."""
    W = lh.weight(lat0)
    M = SamplingMetric(cf, lat0, W)
    sseq = seed_seq.spawn(n_samples)
    if mirror:
        sseq = [s for s in sseq for _ in range(2)]
    res, negs, y = [], [], None
    sqw = np.sqrt(W)
    iters = 0
    for i, ss in enumerate(sseq):
        neg = mirror and (i % 2 != 0)
        if not neg or y is None:
            rng = np.random.default_rng(ss)
            s = {k: rng.normal(0., 1., np.shape(lat0[k])) for k in _keys(lat0)}
            n = rng.normal(0., 1., W.shape)
            nj = cf.vjp(lat0, sqw * n)
            nj = {k: np.reshape(nj[k], np.shape(s[k])) for k in _keys(s)}
            b = axpy(1., nj, s)
            jwj = cf.vjp(lat0, W * cf.jvp(lat0, s))
            grad = {k: np.reshape(jwj[k], np.shape(s[k])) - nj[k] for k in _keys(s)}
            x, st, it = conjugate_gradient(M, s, b, ctl_factory(), grad=grad, nreset=nreset)
            iters += it
            y = b
            yi = x
        res.append(yi)
        negs.append(neg)
    return res, negs, iters
