"""Oracle: geoVI sample drawing (MGVI linear draw + NewtonCG refinement) for a
correlated field under a whitened Gaussian likelihood.  TEST INFRASTRUCTURE
ONLY (tests/, bench.py's cpu_baseline leg).

Restates
  draw_samples, geometric branch        src/minimization/kl_energies.py:103-158
  SamplingEnabler.special_draw_sample   src/operators/sampling_enabler.py:64-86
  DescentMinimizer.__call__             src/minimization/descent_minimizers.py:52-108
  NewtonCG.get_descent_direction        src/minimization/descent_minimizers.py:187-206
  LineSearch (strong Wolfe + zoom)      src/minimization/line_search.py:147-420
  EnergyAdapter(nanisinf=True)          src/minimization/energy_adapter.py:56-92
on latent dicts {key: ndarray} in sorted-key order.  The whitened likelihood
map f (GaussianEnergy(data, 1/var).get_transformation composed with the
response, energy_operators.py:186-195,578-579) is `LOSWhitened` (sigmoid o
LOSResponse, config C3), `GaussWhitened` (GeometryRemover) or
`PoissonWhitened` (exp signal, Poisson counts, config C2).  The geoVI
energy of a sample is 0.5 |T(x) - m|^2 with T = 1 + J0^T f (kl_energies.py:
117-118,147-151); its gradient is (1 + J(x)^T J0) (T(x) - m) and its metric
(1 + J(x)^T J0)(1 + J0^T J(x)).
"""
import numpy as np

from .sampling import AbsDeltaCtl, GradNormCtl, _keys, axpy, conjugate_gradient, vdot


def _shape_like(g, x):
    return {k: np.reshape(g[k], np.shape(x[k])) for k in _keys(x)}


class GaussWhitened:
    """f(x) = sqrt(1/var) cf(x) (GeometryRemover response)"""

    def __init__(self, cf, noise_var):
        self.cf, self.sq = cf, np.sqrt(1. / noise_var)
        self.data_shape = cf.shape

    def f(self, x):
        return self.sq * self.cf.value(x)

    def jvp(self, x, t):
        return self.sq * self.cf.jvp(x, t)

    def vjp(self, x, g):
        return _shape_like(self.cf.vjp(x, self.sq * g), x)


class PoissonWhitened:
    """f(x) = 2 sqrt(lambda), lambda = exp(cf(x)) (PoissonianEnergy
    .get_transformation, energy_operators.py:624-625, composed with the exp
    signal): f = 2 exp(cf / 2), f' = exp(cf / 2)"""

    def __init__(self, cf):
        self.cf = cf
        self.data_shape = cf.shape
        self._cache = (None, None)

    def _h(self, x):
        if self._cache[0] is not x:
            self._cache = (x, np.exp(0.5 * self.cf.value(x)))
        return self._cache[1]

    def f(self, x):
        return 2. * self._h(x)

    def jvp(self, x, t):
        return self._h(x) * self.cf.jvp(x, t)

    def vjp(self, x, g):
        return _shape_like(self.cf.vjp(x, self._h(x) * g), x)


class LOSWhitened:
    """f(x) = sqrt(1/var) R sigmoid(cf(x)), sigmoid = 0.5 + 0.5 tanh
    (pointwise.py:148); R the float32-weight COO matrix of LOSResponse
    (los_response.py:197-233) applied with scipy.sparse"""

    def __init__(self, cf, rows, cols, wgt, nlos, noise_var):
        import scipy.sparse
        self.cf = cf
        self.R = scipy.sparse.coo_matrix((wgt, (rows, cols)), shape=(nlos, int(np.prod(cf.shape)))).tocsr()
        self.RT = self.R.T.tocsr()
        self.sq = np.sqrt(1. / noise_var)
        self.data_shape = (nlos,)
        self._cache = (None, None)

    def _dsig(self, x):
        if self._cache[0] is not x:
            t = np.tanh(self.cf.value(x))
            self._cache = (x, (0.5 + 0.5 * t, 0.5 * (1. - t * t)))
        return self._cache[1]

    def f(self, x):
        sig, _ = self._dsig(x)
        return self.sq * (self.R @ sig.ravel())

    def jvp(self, x, t):
        _, ds = self._dsig(x)
        return self.sq * (self.R @ (ds * self.cf.jvp(x, t)).ravel())

    def vjp(self, x, g):
        _, ds = self._dsig(x)
        v = ds * (self.RT @ (self.sq * g)).reshape(self.cf.shape)
        return _shape_like(self.cf.vjp(x, v), x)


class GeoEnergy:
    """EnergyAdapter(pos, GaussianEnergy(m) @ transformation, nanisinf=True)
    of one sample; value / gradient at a latent position"""

    def __init__(self, lh, x0, m, x):
        self.lh, self.x0, self.m, self.x = lh, x0, m, x
        with np.errstate(all="ignore"):
            fx = lh.f(x)
            self.r = axpy(-1., m, axpy(1., x, _shape_like(lh.vjp(x0, fx), x)))
            v = 0.5 * vdot(self.r, self.r)
        self.value = np.inf if np.isnan(v) else v
        self._grad = None

    @property
    def gradient(self):
        if self._grad is None:
            with np.errstate(all="ignore"):
                lh, x = self.lh, self.x
                self._grad = axpy(1., self.r, lh.vjp(x, lh.jvp(self.x0, self.r)))
        return self._grad

    def metric(self, v):
        lh, x, x0 = self.lh, self.x, self.x0
        u = axpy(1., v, lh.vjp(x0, lh.jvp(x, v)))
        return axpy(1., u, lh.vjp(x, lh.jvp(x0, u)))

    def at(self, x):
        return GeoEnergy(self.lh, self.x0, self.m, x)


class LineSearch:
    """Strong-Wolfe line search (line_search.py:147-347) with the reference's
    defaults and preferred_initial_step_size=1 (NewtonCG)."""

    def __init__(self, c1=1e-4, c2=0.9, max_step_size=1e30, max_iterations=100, max_zoom_iterations=100):
        self.c1, self.c2 = c1, c2
        self.max_step_size, self.max_it, self.max_zoom = max_step_size, max_iterations, max_zoom_iterations
        self.trials = []

    @staticmethod
    def _dd(e, pk):
        return vdot(e.gradient, pk)

    def __call__(self, e0, pk, f_km1=None):
        self.trials.append([])
        phi_0 = e0.value
        dphi_0 = self._dd(e0, pk)
        if dphi_0 >= 0:
            return e0, False
        a0, phi_a0, dphi_a0 = 0., phi_0, dphi_0
        a1 = min(1., 0.99 * self.max_step_size)
        it, e1 = 0, None
        while it < self.max_it:
            it += 1
            if a1 == 0:
                return e0, False
            e1 = e0.at(axpy(a1, pk, e0.x))
            self.trials[-1].append(a1)
            phi_a1 = e1.value
            if np.isnan(phi_a1) or np.abs(phi_a1) > 1e100:
                a1 = (a0 + a1) / 2
                continue
            if phi_a1 > phi_0 + self.c1 * a1 * dphi_0 or (phi_a1 >= phi_a0 and it > 1):
                return self._zoom(a0, a1, phi_0, dphi_0, phi_a0, dphi_a0, phi_a1, e0, pk)
            dphi_a1 = self._dd(e1, pk)
            if abs(dphi_a1) <= -self.c2 * dphi_0:
                return e1, True
            if dphi_a1 >= 0:
                return self._zoom(a1, a0, phi_0, dphi_0, phi_a1, dphi_a1, phi_a0, e0, pk)
            a0, a1 = a1, min(2 * a1, self.max_step_size)
            if a1 == self.max_step_size:
                return e1, False
            phi_a0, dphi_a0 = phi_a1, dphi_a1
        return e1, False

    def _zoom(self, lo, hi, phi_0, dphi_0, phi_lo, dphi_lo, phi_hi, e0, pk):
        """line_search.py:251-347"""
        rec = phi_rec = None
        for i in range(self.max_zoom):
            d = hi - lo
            a, b = min(lo, hi), max(lo, hi)
            if i > 0:
                cchk = 0.2 * d
                aj = _cubicmin(lo, phi_lo, dphi_lo, hi, phi_hi, rec, phi_rec)
            if i == 0 or aj is None or aj > b - cchk or aj < a + cchk:
                qchk = 0.1 * d
                aj = _quadmin(lo, phi_lo, dphi_lo, hi, phi_hi)
                if aj is None or aj > b - qchk or aj < a + qchk:
                    aj = lo + 0.5 * d
            ej = e0.at(axpy(aj, pk, e0.x))
            self.trials[-1].append(aj)
            phi_j = ej.value
            if phi_j > phi_0 + self.c1 * aj * dphi_0 or phi_j >= phi_lo:
                rec, phi_rec = hi, phi_hi
                hi, phi_hi = aj, phi_j
            else:
                dphi_j = self._dd(ej, pk)
                if abs(dphi_j) <= -self.c2 * dphi_0:
                    return ej, True
                if dphi_j * d >= 0:
                    rec, phi_rec = hi, phi_hi
                    hi, phi_hi = lo, phi_lo
                else:
                    rec, phi_rec = lo, phi_lo
                lo, phi_lo, dphi_lo = aj, phi_j, dphi_j
        return ej, False


def _cubicmin(a, fa, fpa, b, fb, c, fc):
    """line_search.py:349-391"""
    with np.errstate(divide="raise", over="raise", invalid="raise"):
        try:
            C = fpa
            db, dc = b - a, c - a
            denom = db * db * dc * dc * (db - dc)
            d1 = np.array([[dc * dc, -(db * db)], [-(dc * dc * dc), db * db * db]])
            A, B = d1 @ np.array([fb - fa - C * db, fc - fa - C * dc])
            A /= denom
            B /= denom
            xmin = a + (-B + np.sqrt(B * B - 3 * A * C)) / (3 * A)
        except (ArithmeticError, TypeError):
            return None
    return xmin if np.isfinite(xmin) else None


def _quadmin(a, fa, fpa, b, fb):
    """line_search.py:393-420"""
    with np.errstate(divide="raise", over="raise", invalid="raise"):
        try:
            db = b - a * 1.0
            B = (fb - fa - fpa * db) / (db * db)
            xmin = a - fpa / (2.0 * B)
        except ArithmeticError:
            return None
    return xmin if np.isfinite(xmin) else None


def newton_cg(e, newton_iters, max_cg=200, nreset=20, alpha=0.1, log=None):
    """NewtonCG(GradientNormController(iteration_limit=newton_iters)) on a
    GeoEnergy (descent_minimizers.py:52-108,187-206).  `log` (a dict) gets
    the inner-CG iteration counts and the line-search trial steps."""
    ctl = GradNormCtl(iteration_limit=newton_iters)
    ls = LineSearch()
    gnorm = np.sqrt(vdot(e.gradient, e.gradient))
    if ctl.start(e.value, gnorm) != 1:
        if log is not None:
            log.setdefault("dir", []).append([])
            log.setdefault("trial", []).append([])
        return e
    f_km1 = None
    dirs = []
    while True:
        g = e.gradient
        if np.sqrt(vdot(g, g)) == 0:
            break
        ic = GradNormCtl(iteration_limit=5) if f_km1 is None else \
            AbsDeltaCtl(alpha * (f_km1 - e.value), iteration_limit=max_cg)
        zero = {k: np.zeros_like(v) for k, v in e.x.items()}
        xs, st, it = conjugate_gradient(e.metric, zero, g, ic, grad={k: -v for k, v in g.items()}, nreset=nreset)
        if st == 2:
            raise ValueError("Cannot find descent direction")
        dirs.append(it)
        pk = {k: -v for k, v in xs.items()}
        new, ok = ls(e, pk, f_km1)
        f_km1 = e.value
        if new.value > e.value:
            break
        if new.value == e.value:
            e = new
            break
        e = new
        if ctl.check(e.value, np.sqrt(vdot(e.gradient, e.gradient))) != 1:
            break
    if log is not None:
        log.setdefault("dir", []).append(dirs)
        log.setdefault("trial", []).append(ls.trials)
    return e


def draw_geovi(lh, x0, n_samples, mirror, seed_seq, lin_ctl_factory, newton_iters, max_cg=200,
               nreset=20, log=None):
    """draw_samples(x0, H, NewtonCG(GradientNormController(newton_iters),
    max_cg_iterations=max_cg), n_samples, mirror) on one rank: returns the
    residual samples (latent dicts) and the total CG iteration count."""
    J0 = lambda t: lh.jvp(x0, t)           # noqa: E731
    J0T = lambda g: lh.vjp(x0, g)          # noqa: E731

    def M(v):
        return axpy(1., v, J0T(J0(v)))
    tmean = axpy(1., x0, J0T(lh.f(x0)))
    sseq = seed_seq.spawn(n_samples)
    if mirror:
        sseq = [s for s in sseq for _ in range(2)]
    res, y, iters = [], None, 0
    lg = log if log is not None else {}
    for i, ss in enumerate(sseq):
        neg = mirror and (i % 2 != 0)
        if not neg or y is None:
            rng = np.random.default_rng(ss)
            s = {k: rng.normal(0., 1., np.shape(x0[k])) for k in _keys(x0)}
            n = rng.normal(0., 1., lh.data_shape)
            nj = J0T(n)
            b = axpy(1., nj, s)
            grad = axpy(-1., nj, J0T(J0(s)))
            xs, st, it = conjugate_gradient(M, s, b, lin_ctl_factory(), grad=grad, nreset=nreset)
            iters += it
            y, yi = b, xs
        sgn = -1. if neg else 1.
        m = axpy(sgn, y, tmean)
        e = GeoEnergy(lh, x0, m, axpy(sgn, yi, x0))
        e = newton_cg(e, newton_iters, max_cg=max_cg, nreset=nreset, log=lg)
        iters += sum(lg["dir"][-1])
        res.append(axpy(-1., x0, e.x))
    return res, iters
