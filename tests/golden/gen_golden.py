"""Generate golden fixtures by importing the reference (NIFTy 8.5) in the
build container.

This script is the ONLY place that touches ``/root/reference``.  It runs here
(the survey/build container), never on the GPU box, and writes small ``.npz``
files next to itself.  Only these data files are committed; the reference
source never leaves the container.

Usage:  python tests/golden/gen_golden.py

Harness shim: ``np.asfarray`` was removed in NumPy 2 but is still called by the
reference (``src/utilities.py:397``, ``src/operators/normal_operators.py:48``);
it is monkey-patched before import.
"""
import os
import sys

import numpy as np

np.asfarray = lambda a, dtype=np.float64: np.asarray(a, dtype=dtype)  # noqa: E731
sys.path.insert(0, "/root/reference")
import nifty8 as ift  # noqa: E402
from nifty8 import ducc_dispatch  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))

CF_ARGS = dict(offset_mean=0, offset_std=(1e-3, 1e-6), fluctuations=(1., 0.8),
               loglogavgslope=(-3., 1), flexibility=(2, 1.), asperity=(0.5, 0.4))


def _save(name, d):
    np.savez_compressed(os.path.join(OUT, name), **d)
    tot = sum(v.nbytes for v in d.values() if isinstance(v, np.ndarray))
    print(f"{name}: {len(d)} arrays, {tot/1e6:.2f} MB raw")


def _flat(mf):
    """MultiField -> dict of arrays with 'key' prefix, sorted keys."""
    return {k: np.asarray(mf[k].val) for k in sorted(mf.keys())}


def gen_dispatch():
    """ducc_dispatch.hartley/fftn/ifftn/vdot (src/ducc_dispatch.py:38-58)."""
    rng = np.random.default_rng(1234)
    cases = [((16,), (0,)), ((7,), (0,)), ((19,), (0,)), ((12, 46), (0, 1)),
             ((12, 9), (0, 1)), ((15, 12), (0, 1)), ((1, 2, 3, 6), (0, 1, 2, 3)),
             ((64, 64), (0, 1)), ((16, 16, 16), (0, 1, 2)), ((128, 128), (0, 1)),
             ((32, 4, 4, 5, 6), (0,)), ((32, 4, 4, 5, 6), (1, 2)),
             ((32, 4, 4, 5, 6), (3, 4)), ((6, 64), (1,)), ((64, 6), (0,)),
             ((8, 12, 10), (0, 2)), ((30, 21), (0, 1)), ((256,), (0,)),
             ((2, 1024), (1,)), ((48, 32, 8), (0, 1, 2))]
    d = {}
    for i, (shp, axes) in enumerate(cases):
        x = rng.standard_normal(shp)
        d[f"c{i}_shape"] = np.array(shp)
        d[f"c{i}_axes"] = np.array(axes)
        d[f"c{i}_x"] = x
        ift.config.update("hartley_convention", "non_canonical_hartley")
        d[f"c{i}_h_nc"] = ducc_dispatch.hartley(x, axes=axes)
        ift.config.update("hartley_convention", "canonical_hartley")
        d[f"c{i}_h_c"] = ducc_dispatch.hartley(x, axes=axes)
        ift.config.update("hartley_convention", "non_canonical_hartley")
        x32 = x.astype(np.float32)
        d[f"c{i}_h32_nc"] = ducc_dispatch.hartley(x32, axes=axes)
        z = x + 1j * rng.standard_normal(shp)
        d[f"c{i}_z"] = z
        d[f"c{i}_fft"] = ducc_dispatch.fftn(z, axes=axes)
        d[f"c{i}_ifft"] = ducc_dispatch.ifftn(z, axes=axes)
        y = rng.standard_normal(shp)
        d[f"c{i}_y"] = y
        d[f"c{i}_vdot"] = np.array(ducc_dispatch.vdot(x, y))
    d["ncases"] = np.array(len(cases))
    _save("dispatch.npz", d)


def gen_geometry():
    """RGSpace/PowerSpace (src/domains/rg_space.py:105-150, power_space.py:155-198)."""
    spaces = [((32, 32), None), ((128, 128), None), ((16, 16, 16), None),
              ((17, 38), (0.99, 1340)), ((64,), None), ((12, 46), (.2, .3)),
              ((7,), 0.2), ((9, 10, 11), (0.5, 0.3, 0.2))]
    d = {}
    for i, (shp, dist) in enumerate(spaces):
        h = ift.RGSpace(shp, distances=dist, harmonic=True)
        ps = ift.PowerSpace(h)
        d[f"s{i}_shape"] = np.array(shp)
        d[f"s{i}_dist"] = np.array(h.distances)
        d[f"s{i}_klen"] = h.get_k_length_array().val
        d[f"s{i}_uniq"] = h.get_unique_k_lengths()
        d[f"s{i}_pindex"] = ps.pindex
        d[f"s{i}_k_lengths"] = ps.k_lengths
        d[f"s{i}_dvol"] = ps.dvol
        pos = h.get_default_codomain()
        d[f"s{i}_pos_dist"] = np.array(pos.distances)
        pd = ift.PowerDistributor(h, ps)
        rng = np.random.default_rng(i)
        v = rng.standard_normal(ps.shape)
        g = rng.standard_normal(h.shape)
        d[f"s{i}_pd_in"] = v
        d[f"s{i}_pd_times"] = pd(ift.makeField(ps, v)).val
        d[f"s{i}_pd_adj_in"] = g
        d[f"s{i}_pd_adj"] = pd.adjoint(ift.makeField(h, g)).val
    d["nspaces"] = np.array(len(spaces))
    _save("geometry.npz", d)


def _cf_case(shape, args, seed, prefix=""):
    """SimpleCorrelatedField forward/Jacobian/adjoint at a fixed point
    (src/library/correlated_fields_simple.py:38-170)."""
    pos_space = ift.RGSpace(shape)
    cf = ift.SimpleCorrelatedField(pos_space, **args, prefix=prefix)
    d = {}
    with ift.random.Context(seed):
        x = ift.from_random(cf.domain, "normal")
        t = ift.from_random(cf.domain, "normal")
        g = ift.from_random(cf.target, "normal")
    lin = cf(ift.Linearization.make_var(x))
    for k, v in _flat(x).items():
        d["x_" + k] = v
    for k, v in _flat(t).items():
        d["t_" + k] = v
    d["g"] = g.val
    d["val"] = lin.val.val
    d["jt"] = lin.jac(t).val
    for k, v in _flat(lin.jac.adjoint(g)).items():
        d["ja_" + k] = v
    d["amp"] = cf.amplitude.force(x).val
    d["pspec"] = cf.power_spectrum.force(x).val
    return d, cf, x


def gen_cf():
    d, _, _ = _cf_case((128, 128), CF_ARGS, 11)
    _save("cf128.npz", d)
    args = dict(offset_mean=1.5, offset_std=None, fluctuations=(0.5, 0.2),
                loglogavgslope=(-2., 0.5), flexibility=None, asperity=None)
    d, _, _ = _cf_case((32, 32), args, 12, prefix="p_")
    _save("cf32_noflex.npz", d)
    args = dict(CF_ARGS)
    args["asperity"] = None
    d, _, _ = _cf_case((16, 16, 16), args, 13)
    _save("cf16cube.npz", d)
    d, _, _ = _cf_case((48, 20), CF_ARGS, 14)
    _save("cf48x20.npz", d)


def _gaussian_problem(n, seed=27, noise=0.01):
    pos_space = ift.RGSpace((n, n))
    cf = ift.SimpleCorrelatedField(pos_space, **CF_ARGS)
    R = ift.GeometryRemover(pos_space)
    sr = R @ cf
    N = ift.ScalingOperator(R.target, noise, np.float64)
    ift.random.push_sseq_from_seed(seed)
    mock = ift.from_random(sr.domain, "normal")
    data = sr(mock) + N.draw_sample()
    lh = ift.GaussianEnergy(data, inverse_covariance=N.inverse) @ sr
    pos = 0.1 * ift.from_random(sr.domain, "normal")
    ift.random.pop_sseq()
    return cf, lh, data, mock, pos


def gen_metric_and_cg():
    """Sampling metric 1 + J^T N^-1 J and CG traces
    (kl_energies.py:115-123, conjugate_gradient.py:48-126)."""
    from nifty8.minimization.quadratic_energy import QuadraticEnergy
    cf, lh, data, mock, pos = _gaussian_problem(128)
    d = {"data": data.val}
    for k, v in _flat(mock).items():
        d["mock_" + k] = v
    for k, v in _flat(pos).items():
        d["pos_" + k] = v
    dtype, f_lh = lh.get_transformation()
    fl = f_lh(ift.Linearization.make_var(pos))
    met = ift.SandwichOperator.make(fl.jac, ift.ScalingOperator(f_lh.target, 1., dtype)) \
        + ift.ScalingOperator(fl.domain, 1., float)
    with ift.random.Context(99):
        v = ift.from_random(fl.domain, "normal")
        b = ift.from_random(fl.domain, "normal")
    for k, val in _flat(v).items():
        d["v_" + k] = val
    for k, val in _flat(b).items():
        d["b_" + k] = val
    for k, val in _flat(met(v)).items():
        d["mv_" + k] = val
    d["flval"] = fl.val.val
    # CG from x0 = 0, fixed iteration counts (nreset crossing at 20)
    for k_it in (1, 5, 25):
        ic = ift.GradientNormController(iteration_limit=k_it)
        ic.enable_logging()
        en = QuadraticEnergy(0 * b, met, b)
        en, st = ift.ConjugateGradient(ic)(en)
        for kk, val in _flat(en.position).items():
            d[f"cg{k_it}_" + kk] = val
        d[f"cg{k_it}_value"] = np.array(en.value)
        d[f"cg{k_it}_status"] = np.array(st)
        d[f"cg{k_it}_hist"] = np.array(ic.history._lst)
    _save("metric128.npz", d)


def gen_draw_samples():
    """MGVI draw for config C1 (128^2, Gaussian, n_samples=2 mirrored, seed 27)
    and a small geoVI draw (kl_energies.py:90-158)."""
    cf, lh, data, mock, pos = _gaussian_problem(128)
    d = {}
    for name, ic in (("short", ift.GradientNormController(iteration_limit=8)),
                     ("fixed", ift.GradientNormController(iteration_limit=20)),
                     ("absdelta", ift.AbsDeltaEnergyController(deltaE=0.05, iteration_limit=100))):
        ic.enable_logging()
        H = ift.StandardHamiltonian(lh, ic)
        ift.random.push_sseq_from_seed(27)
        sl = ift.minimization.kl_energies.draw_samples(pos, H, None, 2, True)
        ift.random.pop_sseq()
        for i, (r, neg) in enumerate(zip(sl._r, sl._n)):
            for k, v in _flat(r).items():
                d[f"{name}_r{i}_" + k] = v
            d[f"{name}_neg{i}"] = np.array(neg)
        d[f"{name}_niter"] = np.array(len(ic.history._lst))
    _save("mgvi128.npz", d)

    # geoVI on 32x32 (small, exercises NewtonCG + line search)
    cf, lh, data, mock, pos = _gaussian_problem(32)
    dd = {"data": data.val}
    for k, v in _flat(pos).items():
        dd["pos_" + k] = v
    ic = ift.AbsDeltaEnergyController(deltaE=0.05, iteration_limit=100)
    H = ift.StandardHamiltonian(lh, ic)
    mini = ift.NewtonCG(ift.AbsDeltaEnergyController(deltaE=0.5, convergence_level=2,
                                                     iteration_limit=5))
    ift.random.push_sseq_from_seed(27)
    sl = ift.minimization.kl_energies.draw_samples(pos, H, mini, 1, True)
    ift.random.pop_sseq()
    for i, r in enumerate(sl._r):
        for k, v in _flat(r).items():
            dd[f"r{i}_" + k] = v
    _save("geovi32.npz", dd)

    # short, rounding-stable variant: 6 linear CG steps, one Newton step with
    # its first-step inner CG (GradientNormController(iteration_limit=5))
    dd = {"data": data.val}
    for k, v in _flat(pos).items():
        dd["pos_" + k] = v
    H = ift.StandardHamiltonian(lh, ift.GradientNormController(iteration_limit=6))
    mini = ift.NewtonCG(ift.GradientNormController(iteration_limit=1))
    ift.random.push_sseq_from_seed(31)
    sl = ift.minimization.kl_energies.draw_samples(pos, H, mini, 1, True)
    ift.random.pop_sseq()
    for i, r in enumerate(sl._r):
        for k, v in _flat(r).items():
            dd[f"r{i}_" + k] = v
    # the MGVI (linear) residuals of the same draw, for the linear stage alone
    ift.random.push_sseq_from_seed(31)
    sl = ift.minimization.kl_energies.draw_samples(pos, H, None, 1, True)
    ift.random.pop_sseq()
    for i, r in enumerate(sl._r):
        for k, v in _flat(r).items():
            dd[f"lin{i}_" + k] = v
    _save("geovi32_short.npz", dd)


def gen_poisson():
    """Config C2 flavour (exp(cf), Poisson counts) at 64^2
    (energy_operators.py:586-625)."""
    pos_space = ift.RGSpace((64, 64))
    cf = ift.SimpleCorrelatedField(pos_space, **CF_ARGS)
    sig = cf.exp()
    ift.random.push_sseq_from_seed(27)
    mock = ift.from_random(sig.domain, "normal")
    lam = sig(mock).val
    counts = ift.random.current_rng().poisson(lam).astype(np.int64)
    data = ift.makeField(pos_space, counts)
    lh = ift.PoissonianEnergy(data) @ sig
    pos = 0.1 * ift.from_random(sig.domain, "normal")
    ift.random.pop_sseq()
    d = {"counts": counts}
    for k, v in _flat(pos).items():
        d["pos_" + k] = v
    dtype, f_lh = lh.get_transformation()
    fl = f_lh(ift.Linearization.make_var(pos))
    d["flval"] = fl.val.val
    met = ift.SandwichOperator.make(fl.jac, ift.ScalingOperator(f_lh.target, 1., dtype)) \
        + ift.ScalingOperator(fl.domain, 1., float)
    with ift.random.Context(5):
        v = ift.from_random(fl.domain, "normal")
    for k, val in _flat(v).items():
        d["v_" + k] = val
    for k, val in _flat(met(v)).items():
        d["mv_" + k] = val
    d["energy"] = np.array(lh(pos).val)
    ic = ift.GradientNormController(iteration_limit=6)
    H = ift.StandardHamiltonian(lh, ic)
    ift.random.push_sseq_from_seed(3)
    sl = ift.minimization.kl_energies.draw_samples(pos, H, None, 1, True)
    ift.random.pop_sseq()
    for i, r in enumerate(sl._r):
        for k, val in _flat(r).items():
            d[f"r{i}_" + k] = val
    _save("poisson64.npz", d)


def gen_los_metric():
    """Config C3 flavour (sigmoid(cf) observed through LOSResponse, Gaussian
    noise) at 64^2 with 300 lines of sight: sampling-metric matvec and short
    MGVI / geoVI draws (kl_energies.py:64-133)."""
    pos_space = ift.RGSpace((64, 64))
    cf = ift.SimpleCorrelatedField(pos_space, **CF_ARGS)
    signal = ift.sigmoid(cf)
    ift.random.push_sseq_from_seed(27)
    rng = ift.random.current_rng()
    starts = rng.random((300, 2)).T
    ends = rng.random((300, 2)).T
    R = ift.LOSResponse(pos_space, starts=list(starts), ends=list(ends))
    sr = R(signal)
    N = ift.ScalingOperator(R.target, 1e-3, np.float64)
    mock = ift.from_random(sr.domain, "normal")
    data = sr(mock) + N.draw_sample()
    pos = 0.1 * ift.from_random(sr.domain, "normal")
    ift.random.pop_sseq()
    lh = ift.GaussianEnergy(data, inverse_covariance=N.inverse) @ sr
    d = {"starts": starts, "ends": ends, "data": data.val}
    for k, v in _flat(pos).items():
        d["pos_" + k] = v
    dtype, f_lh = lh.get_transformation()
    fl = f_lh(ift.Linearization.make_var(pos))
    met = ift.SandwichOperator.make(fl.jac, ift.ScalingOperator(f_lh.target, 1., dtype)) \
        + ift.ScalingOperator(fl.domain, 1., float)
    with ift.random.Context(5):
        v = ift.from_random(fl.domain, "normal")
    for k, val in _flat(v).items():
        d["v_" + k] = val
    for k, val in _flat(met(v)).items():
        d["mv_" + k] = val
    H = ift.StandardHamiltonian(lh, ift.GradientNormController(iteration_limit=6))
    ift.random.push_sseq_from_seed(31)
    sl = ift.minimization.kl_energies.draw_samples(pos, H, None, 1, True)
    ift.random.pop_sseq()
    for i, r in enumerate(sl._r):
        for k, val in _flat(r).items():
            d[f"lin{i}_" + k] = val
    mini = ift.NewtonCG(ift.GradientNormController(iteration_limit=1))
    ift.random.push_sseq_from_seed(31)
    sl = ift.minimization.kl_energies.draw_samples(pos, H, mini, 1, True)
    ift.random.pop_sseq()
    for i, r in enumerate(sl._r):
        for k, val in _flat(r).items():
            d[f"r{i}_" + k] = val
    _save("losmetric64.npz", d)


def gen_los():
    """LOSResponse construction + matvec/rmatvec (los_response.py:34-233)."""
    d = {}
    for i, (shp, nlos) in enumerate((((64, 64), 200), ((40, 24), 50), ((12, 10, 8), 30))):
        space = ift.RGSpace(shp)
        rng = np.random.default_rng(100 + i)
        starts = rng.random((len(shp), nlos))
        ends = rng.random((len(shp), nlos))
        R = ift.LOSResponse(space, starts=list(starts), ends=list(ends))
        coo = R._smat.A  # the underlying scipy coo_matrix
        x = rng.standard_normal(shp)
        y = rng.standard_normal(nlos)
        d[f"l{i}_shape"] = np.array(shp)
        d[f"l{i}_starts"] = starts
        d[f"l{i}_ends"] = ends
        d[f"l{i}_row"] = coo.row.astype(np.int32)
        d[f"l{i}_col"] = coo.col.astype(np.int32)
        d[f"l{i}_wgt"] = coo.data
        d[f"l{i}_x"] = x
        d[f"l{i}_y"] = y
        d[f"l{i}_Rx"] = R(ift.makeField(space, x)).val
        d[f"l{i}_Rty"] = R.adjoint(ift.makeField(R.target, y)).val
    _save("los.npz", d)


def gen_random():
    """RNG stream order: from_random on a MultiDomain draws keys in sorted
    order (multi_field.py:103-127); spawn_sseq children (random.py:114-133)."""
    dom = ift.makeDomain({"zeta": ift.RGSpace(5), "alpha": ift.RGSpace((2, 3)),
                          "mid": ift.DomainTuple.scalar_domain()})
    d = {}
    with ift.random.Context(7):
        mf = ift.from_random(dom, "normal", std=2.)
    for k, v in _flat(mf).items():
        d["mf_" + k] = v
    ift.random.push_sseq_from_seed(27)
    ss = ift.random.spawn_sseq(3)
    for i, s in enumerate(ss):
        with ift.random.Context(s):
            d[f"child{i}"] = ift.random.current_rng().standard_normal(4)
    ift.random.pop_sseq()
    _save("random.npz", d)


KL_CASES = (((), ()), (("fluctuations", "zeromode"), ()), ((), ("loglogavgslope", "spectrum")),
            (("fluctuations", "zeromode"), ("zeromode", "asperity")), (("xi",), ("xi",)))


def gen_kl_constants():
    """SampledKLEnergy with constants / point estimates / invariants
    (kl_energies.py:161-356, sample_list.py:486-507) on the 32^2 Gaussian
    problem: MGVI (6 CG steps) and geoVI (one short Newton step), one mirrored
    pair, seed 41.  Records the KL position keys, value, gradient and the
    residual samples."""
    cf, lh, data, mock, pos = _gaussian_problem(32)
    d = {"data": data.val}
    for k, v in _flat(pos).items():
        d["pos_" + k] = v
    # the reference's own rounding sensitivity: the same draw at an expansion
    # point whose xi is perturbed by 1e-15 (relative); tests allow 10x this
    pos_p = ift.MultiField.from_dict({k: (v * (1 + 1e-15) if k == "xi" else v) for k, v in pos.items()})

    def _rel(a, b):
        return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)

    for ci, (cst, pe) in enumerate(KL_CASES):
        for geo in (False, True):
            kls = []
            for p in (pos, pos_p):
                H = ift.StandardHamiltonian(lh, ift.GradientNormController(iteration_limit=6))
                mini = ift.NewtonCG(ift.GradientNormController(iteration_limit=1)) if geo else None
                ift.random.push_sseq_from_seed(41)
                kls.append(ift.SampledKLEnergy(p, H, 1, mini, True, constants=list(cst),
                                               point_estimates=list(pe)))
                ift.random.pop_sseq()
            kl, klp = kls
            tag = f"c{ci}{'g' if geo else 'm'}_"
            d[tag + "sens_grad"] = np.array(max(_rel(klp.gradient[k].val, kl.gradient[k].val)
                                                for k in kl.gradient.keys()))
            d[tag + "sens_samples"] = np.array(max(
                _rel(klp.samples.local_item(i)[k].val, kl.samples.local_item(i)[k].val)
                for i in range(kl.samples.n_samples) for k in pos.keys() if k != "xi" or "xi" not in pe))
            d[tag + "value"] = np.array(kl.value)
            d[tag + "keys"] = np.array(sorted(kl.position.keys()))
            for k, v in _flat(kl.gradient).items():
                d[tag + "grad_" + k] = v
            sl = kl.samples
            for i in range(sl.n_samples):
                for k, v in _flat(sl.local_item(i)).items():
                    d[tag + f"s{i}_" + k] = v
    _save("kl32_constants.npz", d)


def gen_napprox_probe():
    """The napprox32 geoVI draw's mirrored sample (seed 43, napprox=3): its
    line search meets inf energies at alpha = 1 and 0.5, then zooms.  At the
    zoom's first accepted-side point (alpha_lo ~ 0.0334) the reference's
    directional derivative (LineEnergy.directional_derivative,
    line_search.py:68-74) is compared with a central finite difference of its
    own energies along the same line (h = 1e-7): they disagree by 2.4x, which
    is what sends the reference's zoom to bisection (line_search.py:309-317)
    where a consistent derivative gives a cubic step."""
    from nifty8.minimization import line_search
    LE = line_search.LineEnergy
    zero = []
    orig_init = LE.__init__

    def init(self, line_position, energy, line_direction, offset=0.):
        orig_init(self, line_position, energy, line_direction, offset)
        if line_position == 0.0 and offset == 0.0:
            zero.append(self)
    LE.__init__ = init
    try:
        _, lh, data, _, pos = _gaussian_problem(32)
        H = ift.StandardHamiltonian(lh, ift.GradientNormController(iteration_limit=6))
        mini = ift.NewtonCG(ift.GradientNormController(iteration_limit=1))
        ift.random.push_sseq_from_seed(43)
        ift.minimization.kl_energies.draw_samples(pos, H, mini, 1, True, napprox=3)
        ift.random.pop_sseq()
    finally:
        LE.__init__ = orig_init
    le0 = zero[-1]          # the mirrored sample's (last) line search
    d = {}
    alphas = np.array([0.0, 0.03336566092948427])
    h = 1e-7
    d["alpha"] = alphas
    d["dd"] = np.array([le0.at(a).directional_derivative if a else le0.directional_derivative for a in alphas])
    d["fd"] = np.array([(le0.at(a + h).value - le0.at(a - h).value) / (2 * h) for a in alphas])
    d["value"] = np.array([le0.at(a).value if a else le0.value for a in alphas])
    print("napprox probe: alpha", alphas, "dd", d["dd"], "fd", d["fd"])
    _save("napprox32_probe.npz", d)


def gen_napprox():
    """draw_samples with the napprox diagonal preconditioner
    (kl_energies.py:127-128, probing.py:142-152): MGVI and geoVI on the 32^2
    Gaussian problem, napprox=3, seed 43, 6 preconditioned CG steps."""
    cf, lh, data, mock, pos = _gaussian_problem(32)
    d = {}
    pos_p = ift.MultiField.from_dict({k: (v * (1 + 1e-15) if k == "xi" else v) for k, v in pos.items()})
    for geo in (False, True):
        sls = []
        for p in (pos, pos_p):
            H = ift.StandardHamiltonian(lh, ift.GradientNormController(iteration_limit=6))
            mini = ift.NewtonCG(ift.GradientNormController(iteration_limit=1)) if geo else None
            ift.random.push_sseq_from_seed(43)
            sls.append(ift.minimization.kl_energies.draw_samples(p, H, mini, 1, True, napprox=3))
            ift.random.pop_sseq()
        sl = sls[0]
        tag = "g_" if geo else "m_"
        # the reference's own change under a 1e-15 perturbation of xi
        d[tag + "sens"] = np.array(max(
            np.linalg.norm(b[k].val - a[k].val) / max(np.linalg.norm(a[k].val), 1e-300)
            for a, b in zip(sls[0]._r, sls[1]._r) for k in pos.keys()))
        for i, (r, neg) in enumerate(zip(sl._r, sl._n)):
            for k, v in _flat(r).items():
                d[tag + f"r{i}_" + k] = v
            d[tag + f"neg{i}"] = np.array(neg)
    # the preconditioner diagonal itself (MGVI metric, same seed)
    H = ift.StandardHamiltonian(lh, ift.GradientNormController(iteration_limit=6))
    ift.random.push_sseq_from_seed(43)
    met = H(ift.Linearization.make_var(pos, want_metric=True)).metric
    diag = ift.probing.approximation2endo(met, 3)
    ift.random.pop_sseq()
    for k, v in _flat(diag).items():
        d["diag_" + k] = v
    _save("napprox32.npz", d)


class _Tracer:
    """Records the decisions of one draw_samples call of the reference by
    wrapping (in this process only) ConjugateGradient.__call__ (every
    controller check: iteration number and energy value),
    DescentMinimizer.__call__ (one NewtonCG refinement per sample) and
    LineEnergy.at (every trial step of the line search).

    events[s] for refinement sample s (draw order):
      "lin"   energies of the linear sampling CG that produced its pair
      "newton" energies at the outer controller checks
      "dir"   list (per Newton step) of inner-CG energy lists
      "trial" list (per Newton step) of line-search trial step sizes"""

    def __init__(self, lin_ctl):
        from nifty8.minimization import conjugate_gradient, descent_minimizers, line_search
        self.mods = (conjugate_gradient.ConjugateGradient, descent_minimizers.DescentMinimizer,
                     line_search.LineEnergy)
        self.lin_ctl = lin_ctl
        self.lin = []          # one energy list per linear solve
        self.samples = []      # one dict per refinement
        self.orig = None

    def __enter__(self):
        CG, DM, LE = self.mods
        self.orig = (CG.__call__, DM.__call__, LE.at)
        cg_call, dm_call, le_at = self.orig
        tr = self

        def _watch(ctl, sink):
            chk = ctl.check

            def check(energy):
                st = chk(energy)
                sink.append(float(energy.value))
                return st
            ctl.check = check
            return chk

        def cg(self_, energy, preconditioner=None):
            ctl = self_._controller
            sink = []
            if ctl is tr.lin_ctl:
                tr.lin.append(sink)
            else:
                s = tr.samples[-1]
                s["dir"].append(sink)
                s["trial"].append([])
                s["trialE"].append([])
            chk = _watch(ctl, sink)
            try:
                return cg_call(self_, energy, preconditioner)
            finally:
                ctl.check = chk

        def dm(self_, energy):
            s = {"lin": len(tr.lin) - 1, "newton": [], "dir": [], "trial": [], "trialE": []}
            tr.samples.append(s)
            chk = _watch(self_._controller, s["newton"])
            try:
                return dm_call(self_, energy)
            finally:
                self_._controller.check = chk

        def at(self_, line_position):
            res = le_at(self_, line_position)
            if tr.samples and tr.samples[-1]["trial"]:
                tr.samples[-1]["trial"][-1].append(float(line_position))
                try:
                    v = float(res.value)
                except FloatingPointError:
                    v = np.nan
                tr.samples[-1]["trialE"][-1].append(v)
            return res

        CG.__call__, DM.__call__, LE.at = cg, dm, at
        return self

    def __exit__(self, *a):
        CG, DM, LE = self.mods
        CG.__call__, DM.__call__, LE.at = self.orig


def _pad(lists, fill=np.nan):
    """ragged lists -> 2-D array padded with `fill` (nan; inf where the
    values themselves may be nan)"""
    n = max([len(x) for x in lists] + [1])
    out = np.full((len(lists), n), fill)
    for i, x in enumerate(lists):
        out[i, :len(x)] = x
    return out


def _cube_problem(n=16):
    pos_space = ift.RGSpace((n, n, n))
    cf = ift.SimpleCorrelatedField(pos_space, **dict(CF_ARGS, asperity=None))
    R = ift.GeometryRemover(pos_space)
    sr = R @ cf
    # noise variance 1: the 100-step linear solve converges (at 0.01 it is
    # chaotic from the 16th step on, as the 2-D GeometryRemover cases)
    N = ift.ScalingOperator(R.target, 1.0, np.float64)
    ift.random.push_sseq_from_seed(29)
    mock = ift.from_random(sr.domain, "normal")
    data = sr(mock) + N.draw_sample()
    pos = 0.1 * ift.from_random(sr.domain, "normal")
    ift.random.pop_sseq()
    lh = ift.GaussianEnergy(data, inverse_covariance=N.inverse) @ sr
    return lh, pos, data


def _los_problem(n=64, nlos=300):
    pos_space = ift.RGSpace((n, n))
    cf = ift.SimpleCorrelatedField(pos_space, **CF_ARGS)
    signal = ift.sigmoid(cf)
    ift.random.push_sseq_from_seed(27)
    rng = ift.random.current_rng()
    starts = rng.random((nlos, 2)).T
    ends = rng.random((nlos, 2)).T
    R = ift.LOSResponse(pos_space, starts=list(starts), ends=list(ends))
    sr = R(signal)
    N = ift.ScalingOperator(R.target, 1e-3, np.float64)
    mock = ift.from_random(sr.domain, "normal")
    data = sr(mock) + N.draw_sample()
    pos = 0.1 * ift.from_random(sr.domain, "normal")
    ift.random.pop_sseq()
    lh = ift.GaussianEnergy(data, inverse_covariance=N.inverse) @ sr
    return lh, pos, {"starts": starts, "ends": ends, "data": data.val}


class _FFTNoise:
    """Context: every Hartley transform of the reference's operators
    (harmonic_operators.py:27,211) returns its output times
    (1 + 2^-52 N(0, 1)) elementwise -- the rounding of another, equally
    valid FFT implementation (the build's kernels round differently from
    pocketfft in every matvec, not once at the start)."""

    def __init__(self, seed):
        self.rng = np.random.default_rng(seed)

    def __enter__(self):
        from nifty8.operators import harmonic_operators as ho
        self.ho, self.orig = ho, ho.hartley
        rng, orig = self.rng, self.orig

        def hartley(a, axes=None):
            out = orig(a, axes=axes)
            return out * (1 + 2.0**-52 * rng.standard_normal(out.shape))
        ho.hartley = hartley
        return self

    def __exit__(self, *a):
        self.ho.hartley = self.orig


def _perturbed(pos):
    """three last-bit perturbations of a draw: xi scaled by 1 + 1e-15, and
    two runs with rounding-level noise on every Hartley transform
    (_FFTNoise seeds 1, 2).  Returns [(position, context)]."""
    import contextlib
    p1 = ift.MultiField.from_dict({k: (v * (1 + 1e-15) if k == "xi" else v) for k, v in pos.items()})
    return [(p1, contextlib.nullcontext()), (pos, _FFTNoise(1)), (pos, _FFTNoise(2))]


def _sens(sl, perturbed, pos):
    """largest relative change of any residual sample over the perturbed runs"""
    return max(np.linalg.norm(b[k].val - a[k].val) / max(np.linalg.norm(a[k].val), 1e-300)
               for slp in perturbed for a, b in zip(sl._r, slp._r) for k in pos.keys())


GEOVI_TRACE_CASES = {
    # geovi32.npz: the demo NewtonCG with the AbsDelta inner-CG branch
    "g32": dict(problem="gauss32", seed=27, nsamp=1, lin=("absdelta", 0.05, 100),
                newton=("absdelta", 0.5, 2, 5), max_cg=200),
    # the bench chain (sigmoid o LOS) with the bench's controllers, 2 pairs
    "bench64": dict(problem="los64", seed=1000, nsamp=2, lin=("gradnorm", 100),
                    newton=("gradnorm", 2), max_cg=50),
    # four Newton steps: three AbsDeltaEnergyController(0.1 dE) inner solves
    "newton64": dict(problem="los64", seed=1002, nsamp=1, lin=("gradnorm", 100),
                     newton=("gradnorm", 4), max_cg=50),
    # 3-D: 16^3 CorrelatedField (no asperity), GeometryRemover Gaussian --
    # the 3-D bin fold and the lowered Newton metric at d = 3
    "cube16": dict(problem="cube16", seed=1003, nsamp=2, lin=("gradnorm", 100),
                   newton=("gradnorm", 2), max_cg=50),
    # napprox32.npz's geoVI draw (napprox=3 preconditioner)
    "napprox32": dict(problem="gauss32", seed=43, nsamp=1, lin=("gradnorm", 6),
                      newton=("gradnorm", 1), max_cg=200, napprox=3),
    # the demo controllers of SURVEY §8(d) on the same chain
    "demo64": dict(problem="los64", seed=1001, nsamp=2, lin=("absdelta", 0.05, 100),
                   newton=("absdelta", 0.5, 2, 15), max_cg=200),
}


def _ctl(spec):
    if spec[0] == "gradnorm":
        return ift.GradientNormController(iteration_limit=spec[1])
    if len(spec) == 3:
        return ift.AbsDeltaEnergyController(deltaE=spec[1], iteration_limit=spec[2])
    return ift.AbsDeltaEnergyController(deltaE=spec[1], convergence_level=spec[2], iteration_limit=spec[3])


def gen_geovi_trace():
    """Multi-step geoVI draws with every controller decision recorded
    (descent_minimizers.py:52-108,187-206, iteration_controllers.py:356-423,
    line_search.py:147-250): per sample the linear CG energies, the Newton
    outer energies, every inner-CG energy (first step GradientNormController(5),
    later steps the AbsDeltaEnergyController(0.1 dE) branch) and the line
    search's trial step sizes.  Each case is also run under three last-bit
    perturbations (_perturbed): the reference's own sensitivity."""
    d = {}
    for name, c in GEOVI_TRACE_CASES.items():
        if c["problem"] == "gauss32":
            _, lh, data, _, pos = _gaussian_problem(32)
            d[name + "_data"] = data.val
        elif c["problem"] == "cube16":
            lh, pos, data = _cube_problem()
            d[name + "_data"] = data.val
        else:
            lh, pos, extra = _los_problem()
            for k, v in extra.items():
                d[f"{name}_{k}"] = v
        for k, v in _flat(pos).items():
            d[f"{name}_pos_{k}"] = v
        runs = []
        import contextlib
        for p, ctx in [(pos, contextlib.nullcontext())] + _perturbed(pos):
            ic = _ctl(c["lin"])
            H = ift.StandardHamiltonian(lh, ic)
            mini = ift.NewtonCG(_ctl(c["newton"]), max_cg_iterations=c["max_cg"])
            ift.random.push_sseq_from_seed(c["seed"])
            with _Tracer(ic) as tr, ctx:
                sl = ift.minimization.kl_energies.draw_samples(p, H, mini, c["nsamp"], True,
                                                               napprox=c.get("napprox", 0))
            ift.random.pop_sseq()
            runs.append((sl, tr))
        (sl, tr), pruns = runs[0], runs[1:]
        d[name + "_sens"] = np.array(_sens(sl, [r[0] for r in pruns], pos))
        d[name + "_nsamples"] = np.array(len(sl._r))
        for i, r in enumerate(sl._r):
            for k, v in _flat(r).items():
                d[f"{name}_r{i}_{k}"] = v
        # the unperturbed trace ("") and the perturbed ones ("p1_" ...): the
        # tests hold the build to the reference where the reference agrees
        # with itself
        for pre, t_ in [("", tr)] + [(f"p{j + 1}_", r[1]) for j, r in enumerate(pruns)]:
            d[f"{name}_{pre}lin"] = _pad(t_.lin)
            for i, s in enumerate(t_.samples):
                t = f"{name}_{pre}s{i}_"
                d[t + "lin"] = np.array(s["lin"])
                d[t + "newton"] = np.array(s["newton"])
                d[t + "dir"] = _pad(s["dir"])
                d[t + "trial"] = _pad(s["trial"])
                d[t + "trialE"] = _pad(s["trialE"], fill=np.inf)
            print(name, pre or "base", "linear CG checks", [len(x) for x in t_.lin],
                  "newton checks", [len(s["newton"]) for s in t_.samples],
                  "inner CG checks", [[len(x) for x in s["dir"]] for s in t_.samples])
        d[name + "_nperturbed"] = np.array(len(pruns))
        print(name, "sens", float(d[name + "_sens"]))
    _save("geovi_trace.npz", d)


def gen_mgvi_absdelta_trace():
    """The mgvi128.npz "absdelta" draw (AbsDeltaEnergyController(0.05,
    iteration_limit=100), 128^2, seed 27, 2 mirrored pairs) with the energy of
    every linear-CG check, unperturbed and under three last-bit perturbations
    (_perturbed): the reference's own spread, which bounds the tests."""
    cf, lh, data, mock, pos = _gaussian_problem(128)
    d = {}
    runs = []
    import contextlib
    for p, ctx in [(pos, contextlib.nullcontext())] + _perturbed(pos):
        ic = ift.AbsDeltaEnergyController(deltaE=0.05, iteration_limit=100)
        H = ift.StandardHamiltonian(lh, ic)
        ift.random.push_sseq_from_seed(27)
        with _Tracer(ic) as tr, ctx:
            sl = ift.minimization.kl_energies.draw_samples(p, H, None, 2, True)
        ift.random.pop_sseq()
        runs.append((sl, tr))
    (sl, tr), pruns = runs[0], runs[1:]
    d["sens"] = np.array(_sens(sl, [r[0] for r in pruns], pos))
    d["lin"] = _pad(tr.lin)
    for j, r in enumerate(pruns):
        d[f"p{j + 1}_lin"] = _pad(r[1].lin)
    d["nperturbed"] = np.array(len(pruns))
    print("mgvi absdelta: checks", [len(x) for x in tr.lin], [[len(x) for x in r[1].lin] for r in pruns],
          "sens", float(d["sens"]))
    _save("mgvi128_absdelta_trace.npz", d)


def gen_kl_metric():
    """SampledKLEnergyClass.apply_metric (kl_energies.py:340-350 ->
    sample_list.py:285-310): the sample average of the Hamiltonian's metric
    (likelihood Fisher metric + identity) at every sample position, for a
    fixed ResidualSampleList (two mirrored pairs of seeded residuals at a
    seeded mean) -- no CG inside, so the fixture pins the averaging alone.
    Gaussian (32^2, GeometryRemover) and Poissonian (32^2, exp) likelihoods;
    the KL value / gradient at the same samples alongside."""
    d = {}
    for tag in ("g", "p"):
        pos_space = ift.RGSpace((32, 32))
        cf = ift.SimpleCorrelatedField(pos_space, **CF_ARGS)
        ift.random.push_sseq_from_seed(51)
        if tag == "g":
            R = ift.GeometryRemover(pos_space)
            sr = R @ cf
            N = ift.ScalingOperator(R.target, 0.01, np.float64)
            mock = ift.from_random(sr.domain, "normal")
            data = sr(mock) + N.draw_sample()
            lh = ift.GaussianEnergy(data, inverse_covariance=N.inverse) @ sr
            d[tag + "_data"] = data.val
        else:
            sig = cf.exp()
            mock = ift.from_random(sig.domain, "normal")
            counts = ift.random.current_rng().poisson(sig(mock).val).astype(np.int64)
            lh = ift.PoissonianEnergy(ift.makeField(pos_space, counts)) @ sig
            d[tag + "_counts"] = counts
        mean = 0.1 * ift.from_random(lh.domain, "normal")
        res = [0.3 * ift.from_random(lh.domain, "normal") for _ in range(2)]
        v = ift.from_random(lh.domain, "normal")
        ift.random.pop_sseq()
        H = ift.StandardHamiltonian(lh)
        sl = ift.ResidualSampleList(mean, [res[0], res[0], res[1], res[1]], [False, True, False, True])
        kl = ift.minimization.kl_energies.SampledKLEnergyClass(sl, H, [], None, True)
        for k, val in _flat(mean).items():
            d[f"{tag}_mean_" + k] = val
        for i, r in enumerate(res):
            for k, val in _flat(r).items():
                d[f"{tag}_r{i}_" + k] = val
        for k, val in _flat(v).items():
            d[f"{tag}_v_" + k] = val
        for k, val in _flat(kl.apply_metric(v)).items():
            d[f"{tag}_mv_" + k] = val
        for k, val in _flat(kl.metric(v)).items():
            d[f"{tag}_mop_" + k] = val
        d[tag + "_value"] = np.array(kl.value)
        for k, val in _flat(kl.gradient).items():
            d[f"{tag}_grad_" + k] = val
    _save("klmetric32.npz", d)


def gen_optimize_kl():
    """optimize_kl (optimize_kl.py:51-412) end to end on the 32^2 Gaussian
    problem: 3 global iterations (MGVI, one mirrored pair; then one MAP
    iteration with n_samples = 0; then geoVI, one pair), NewtonCG(2) on the
    KL, no output directory.  Records the mean after every iteration and the
    KL energy history; the reference's own sensitivity to a 1e-15 relative
    perturbation of the initial xi bounds the comparison tolerance."""
    cf, lh, data, mock, pos = _gaussian_problem(32)
    d = {"data": data.val}
    for k, v in _flat(pos).items():
        d["pos_" + k] = v
    pos_p = ift.MultiField.from_dict({k: (v * (1 + 1e-15) if k == "xi" else v) for k, v in pos.items()})
    runs = []
    for p0 in (pos, pos_p):
        means = []
        ift.random.push_sseq_from_seed(61)
        sl, mean = ift.optimize_kl(
            lh, 3, lambda i: 0 if i == 1 else 1,
            ift.NewtonCG(ift.GradientNormController(iteration_limit=2)),
            ift.GradientNormController(iteration_limit=8),
            lambda i: ift.NewtonCG(ift.GradientNormController(iteration_limit=1)) if i == 2 else None,
            initial_position=p0, plot_energy_history=False, plot_minisanity_history=False,
            return_final_position=True, inspect_callback=lambda sl, i: means.append(
                {k: np.asarray(v.val) for k, v in (sl._m if hasattr(sl, "_m") else sl.local_item(0)).items()}))
        ift.random.pop_sseq()
        runs.append((means, sl, mean))
    (means, sl, mean), (means_p, _, _) = runs
    for i, m in enumerate(means):
        for k, v in m.items():
            d[f"it{i}_mean_" + k] = v
        d[f"it{i}_sens"] = np.array(max(np.linalg.norm(means_p[i][k] - v) / max(np.linalg.norm(v), 1e-300)
                                        for k, v in m.items()))
    for k, v in _flat(mean).items():
        d["final_" + k] = v
    for i in range(sl.n_samples):
        for k, v in _flat(sl.local_item(i)).items():
            d[f"s{i}_" + k] = v
    _save("optkl32.npz", d)


FFTOP_CASES = [((16,), 0.1, None), ((12, 9), (0.4, 2.7), None), ((6, 8, 10), (1., 0.5, 3.), None),
               ((10, 14), (0.7, 1.3), "batched")]


def gen_fftop():
    """FFTOperator volume factors and modes (harmonic_operators.py:34-123):
    times / adjoint_times / inverse_times / adjoint_inverse_times from the
    position and from the harmonic side, on RGSpaces with non-unit distances
    and as one space of a product domain."""
    rng = np.random.default_rng(77)
    d = {}
    for i, (shape, dist, kind) in enumerate(FFTOP_CASES):
        sp = ift.RGSpace(shape, distances=dist)
        if kind == "batched":
            dom = ift.DomainTuple.make((ift.UnstructuredDomain(3), sp))
            op = ift.FFTOperator(dom, space=1)
        else:
            dom = ift.DomainTuple.make(sp)
            op = ift.FFTOperator(dom)
        for side, D in (("pos", op.domain), ("harm", op.target)):
            x = rng.standard_normal(D.shape) + 1j * rng.standard_normal(D.shape)
            d[f"c{i}_{side}_x"] = x
            f = ift.makeField(D, x)
            if side == "pos":
                d[f"c{i}_times"] = op.times(f).val
                d[f"c{i}_adjinv"] = op.adjoint_inverse_times(f).val
            else:
                d[f"c{i}_adj"] = op.adjoint_times(f).val
                d[f"c{i}_inv"] = op.inverse_times(f).val
    _save("fftop.npz", d)


def _op_case(op, seed, d, tag):
    """value, Jacobian and adjoint of `op` at a fixed random point"""
    with ift.random.Context(seed):
        x = ift.from_random(op.domain, "normal")
        t = ift.from_random(op.domain, "normal")
        g = ift.from_random(op.target, "normal")
    lin = op(ift.Linearization.make_var(x))
    for k, v in _flat(x).items():
        d[f"{tag}x_" + k] = v
    for k, v in _flat(t).items():
        d[f"{tag}t_" + k] = v
    d[tag + "g"] = g.val
    d[tag + "val"] = lin.val.val
    d[tag + "jt"] = lin.jac(t).val
    for k, v in _flat(lin.jac.adjoint(g)).items():
        d[f"{tag}ja_" + k] = v
    return x


def gen_cfm():
    """CorrelatedFieldMaker (src/library/correlated_fields.py:388-1115):
    a two-component product spectrum (2-D space x 1-D frequency, LogNormal
    zero mode, offset), a single component with a maker prefix distinct from
    the component prefix (the fused lowering), a unit zero mode and a Matern
    component; values, Jacobians, adjoints and normalised amplitudes."""
    d = {}
    sp = ift.RGSpace((24, 20), distances=(0.05, 0.07))
    fr = ift.RGSpace(18, distances=0.3)
    cfm = ift.CorrelatedFieldMaker("pp_")
    cfm.add_fluctuations(sp, (1., 0.4), (1.2, 0.5), (0.6, 0.3), (-3., 0.5), prefix="sp_")
    cfm.add_fluctuations(fr, (0.7, 0.2), (0.9, 0.4), None, (-2., 0.4), prefix="fr_")
    cfm.set_amplitude_total_offset(0.3, (0.8, 0.1))
    op = cfm.finalize(prior_info=0)
    x = _op_case(op, 41, d, "prod_")
    for i, na in enumerate(cfm.get_normalized_amplitudes()):
        d[f"prod_na{i}"] = na.force(x).val
    d["prod_totfl"] = np.asarray(cfm.total_fluctuation.force(x).val)
    for i in range(2):
        d[f"prod_slfl{i}"] = np.asarray(cfm.slice_fluctuation(i).force(x).val)
        d[f"prod_avfl{i}"] = np.asarray(cfm.average_fluctuation(i).force(x).val)

    one = ift.RGSpace((40, 36), distances=(0.02, 0.03))
    cfm = ift.CorrelatedFieldMaker("mk_")
    cfm.add_fluctuations(one, (0.9, 0.3), (1.1, 0.4), (0.5, 0.2), (-2.5, 0.6), prefix="amp_")
    cfm.set_amplitude_total_offset(-0.4, (1e-2, 1e-3))
    op = cfm.finalize(prior_info=0)
    x = _op_case(op, 42, d, "one_")
    d["one_amp"] = cfm.amplitude.force(x).val

    cfm = ift.CorrelatedFieldMaker("u_")
    cfm.add_fluctuations(ift.RGSpace(64), (1., 0.5), None, None, (-3., 1.))
    cfm.set_amplitude_total_offset(0., 1.)
    op = cfm.finalize(prior_info=0)
    x = _op_case(op, 43, d, "unit_")
    d["unit_amp"] = cfm.amplitude.force(x).val

    cfm = ift.CorrelatedFieldMaker("m_")
    cfm.add_fluctuations_matern(ift.RGSpace((32, 32), distances=0.1), (1., 0.3), (2., 0.5), (-3., 0.5))
    cfm.set_amplitude_total_offset(1., (1e-2, 1e-3))
    op = cfm.finalize(prior_info=0)
    x = _op_case(op, 44, d, "mat_")
    d["mat_amp"] = cfm.amplitude.force(x).val
    _save("cfm.npz", d)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        for name in sys.argv[1:]:
            globals()["gen_" + name]()
        sys.exit(0)
    gen_dispatch()
    gen_geometry()
    gen_cf()
    gen_metric_and_cg()
    gen_draw_samples()
    gen_poisson()
    gen_los()
    gen_los_metric()
    gen_random()
    gen_kl_constants()
    gen_napprox()
    gen_cfm()
