"""GPU: the two-phase amplitude kernels (csrc/nft_amp2.hip) -- the
correlated-field amplitude JVP / VJP of src/library/correlated_fields.py:
105-212 (_SlopeRemover, _TwoLogIntegrations, _Normalization) linearised at a
point, in two launches each -- against the ten-kernel path (nft_amp.hip) and
the torch restatement (pinned to the reference by the CF golden tests), and
the CG work they carry for the amplitude keys (direction with the JVP,
update + finalize with the VJP) against the separate CG launches.

Tolerances: JVP / VJP rtol 1e-12 (summation order only); carried CG after 8
and 25 steps rtol 1e-11 against the separate launches (the ill-conditioned
sampling CG amplifies rounding by ~10x per step past ~10 steps, see
test_parity_gpu.py); batched == single bitwise."""
import copy

import numpy as np
import pytest
import torch

from conftest import golden
from test_parity_gpu import CF_ARGS, _los_problem, rel

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ift(dev):
    import nifty_amd
    return nifty_amd


def _toggle(on):
    from nifty_amd import _native
    _native.load().nft_amp2_set_enabled(on)


@pytest.fixture
def restore():
    yield
    _toggle(-1)


CASES = [((2048, 2048), CF_ARGS), ((700, 300), dict(CF_ARGS, asperity=None)),
         ((8192,), dict(CF_ARGS, offset_std=None)), ((96, 96), dict(CF_ARGS, flexibility=None, asperity=None)),
         ((6, 5), CF_ARGS)]


def _close_keys(got, want, tag, rtol=1e-12):
    """cotangents key by key within rtol of the whole cotangent's norm (a
    scalar key is a difference of large sums: its own relative error is the
    cancellation's, in either summation order), and the whole vector"""
    g = np.concatenate([got[k].cpu().numpy().ravel() for k in want])
    w = np.concatenate([want[k].cpu().numpy().ravel() for k in want])
    assert rel(g, w) < rtol, tag
    scale = np.linalg.norm(w)
    for k in want:
        err = np.linalg.norm(got[k].cpu().numpy() - want[k].cpu().numpy())
        assert err <= rtol * scale, (tag, k, err / scale)


def _setup(ift, shape, args, k):
    from nifty_amd.packing import PackedLayout
    cf = ift.SimpleCorrelatedField(ift.RGSpace(shape), **args)
    amp = cf.amp
    keys = list(amp.domain_dict)
    x = ift.from_random(cf.domain, "normal")
    _, c = amp.forward({kk: x[kk].val for kk in keys})
    const, keep = amp.native_const(c)
    lin = amp.forward_native({kk: x[kk].val for kk in keys})
    lay = PackedLayout(cf.domain)
    D = torch.stack([lay.pack(ift.from_random(cf.domain, "normal")) for _ in range(k)])
    off = dict(zip(lay.keys, lay.offsets))
    return cf, amp, keys, c, (const, keep), lin, lay, D, off


@pytest.mark.parametrize("shape,args", CASES)
@pytest.mark.parametrize("k", [1, 3, 4, 5])
def test_amp2_jvp_vjp(ift, restore, shape, args, k):
    cf, amp, keys, c, (const, keep), lin, lay, D, off = _setup(ift, shape, args, k)
    dev = D.device
    B = amp.B
    g = torch.randn((k, B), dtype=torch.float64, device=dev)
    res = {}
    for on in (1, 0):
        _toggle(on)
        for name, cst in (("host", const), ("lin", lin)):
            da = torch.empty((B, k), dtype=torch.float64, device=dev)
            amp.native_jvp_batched(cst, D, off, da, interleave=True)
            Q = torch.zeros_like(D)
            amp.native_vjp_batched(cst, g, Q, off, D, 0.75)
            res[on, name] = (da.clone(), Q.clone())
    for j in range(k):
        tj = {kk: lay.views(D[j])[kk] for kk in keys}
        ref = amp.jvp(c, tj)
        refv = amp.vjp(c, g[j])
        for name in ("host", "lin"):
            da, Q = res[1, name]
            assert rel(da[:, j].cpu().numpy(), ref.cpu().numpy()) < 1e-12, (name, j)
            assert rel(da[:, j].cpu().numpy(), res[0, name][0][:, j].cpu().numpy()) < 1e-12, (name, j)
            qv = lay.views(Q[j])
            _close_keys(qv, {kk: refv[kk].reshape(qv[kk].shape) + 0.75 * tj[kk] for kk in keys}, (name, j))
    # per RHS independent of the batch: row j of a batch == a batch of one
    _toggle(1)
    for name, cst in (("host", const), ("lin", lin)):
        for j in range(k):
            da1 = torch.empty((B, 1), dtype=torch.float64, device=dev)
            amp.native_jvp_batched(cst, D[j:j + 1], off, da1, interleave=True)
            assert torch.equal(da1[:, 0], res[1, name][0][:, j]), (name, j)
            Q1 = torch.zeros_like(D[j:j + 1])
            amp.native_vjp_batched(cst, g[j:j + 1], Q1, off, D[j:j + 1], 0.75)
            assert torch.equal(Q1[0], res[1, name][1][j]), (name, j)


@pytest.mark.parametrize("shape,args", CASES + [((4096, 4096), CF_ARGS)])
def test_amp2_table_bitwise(ift, shape, args, monkeypatch):
    """the constant-scan table (nft_amp2_prepare: the constant tile-local
    scans and tile sums formed once per linearisation) changes no bit of the
    JVP / VJP, for host and device constant sets (bitwise, k = 3)"""
    from nifty_amd.library import correlated_fields_simple as cfs
    with ift.random.Context(23):
        cf, amp, keys, c, (const, keep), lin, lay, D, off = _setup(ift, shape, args, 3)
    g = torch.randn((3, amp.B), dtype=torch.float64, device=D.device,
                    generator=torch.Generator(device=D.device).manual_seed(23))
    res = {}
    for on in (True, False):
        monkeypatch.setattr(cfs, "AMP2_TABLE", on)
        for name, cst in (("host", const), ("lin", lin)):
            assert (amp.amp2_table(cst) is not None) == on
            da = torch.empty((amp.B, 3), dtype=torch.float64, device=D.device)
            amp.native_jvp_batched(cst, D, off, da, interleave=True)
            Q = torch.zeros_like(D)
            amp.native_vjp_batched(cst, g, Q, off, D, 0.75)
            res[on, name] = (da, Q)
    def diff(a, b):
        d = (a - b).abs()
        nz = torch.nonzero(d)
        return float(d.max()), int(nz.shape[0]), nz[:4].tolist()
    for name in ("host", "lin"):
        assert torch.equal(res[True, name][0], res[False, name][0]), (name, diff(res[True, name][0], res[False, name][0]))
        assert torch.equal(res[True, name][1], res[False, name][1]), (name, diff(res[True, name][1], res[False, name][1]))


def test_amp2_table_carried_cg_bitwise(ift, monkeypatch):
    """the carried sampling CG (direction with the JVP, update + finalize with
    the VJP) with and without the constant-scan table: the same iterates
    bitwise after 12 steps"""
    from nifty_amd.library import correlated_fields_simple as cfs
    from nifty_amd.minimization import fused_cg
    cf, lh, pos = _los_problem(ift, golden("losmetric64.npz"))
    dtype, f_lh = lh.get_transformation()
    fl = f_lh(ift.Linearization.make_var(pos))
    A = (ift.SandwichOperator.make(fl.jac, ift.ScalingOperator(f_lh.target, 1., dtype))
         + ift.ScalingOperator(fl.domain, 1., float))
    core, W, shift = fused_cg.fusable_metric(A)
    es = [ift.QuadraticEnergy(0.1 * ift.from_random(cf.domain, "normal"), A, ift.from_random(cf.domain, "normal"))
          for _ in range(3)]
    out = {}
    for on in (True, False):
        monkeypatch.setattr(cfs, "AMP2_TABLE", on)
        cg = fused_cg.FusedCGBatch(core, W, shift, [ift.GradientNormController(iteration_limit=12) for _ in es])
        out[on] = cg.run(es)
        assert cg.path.startswith("carry"), cg.path
    for (e1, s1), (e2, s2) in zip(out[True], out[False]):
        assert s1 == s2
        for key in cf.domain.keys():
            assert torch.equal(e1.position[key].val, e2.position[key].val), key


def test_amp2_per_item_constants(ift, restore):
    """item_consts (one linearisation point per RHS, the batched geoVI
    refinement): every RHS against its own single-point JVP / VJP"""
    cf, amp, keys, c, (const, keep), lin, lay, D, off = _setup(ift, (512, 512), CF_ARGS, 3)
    X = torch.stack([lay.pack(0.3 * ift.from_random(cf.domain, "normal")) for _ in range(3)])
    lb = amp.forward_rows(amp._ptrs(X, off), 3, X.shape[1], X.device)
    B = amp.B
    g = torch.randn((3, B), dtype=torch.float64, device=D.device)
    da = torch.empty((B, 3), dtype=torch.float64, device=D.device)
    amp.native_jvp_batched(lb.host, D, off, da, interleave=True, item_consts=lb.dconst.data_ptr())
    Q = torch.zeros_like(D)
    amp.native_vjp_batched(lb.host, g, Q, off, item_consts=lb.dconst.data_ptr())
    for j in range(3):
        _, cj = amp.forward({kk: lay.views(X[j])[kk] for kk in keys})
        tj = {kk: lay.views(D[j])[kk] for kk in keys}
        assert rel(da[:, j].cpu().numpy(), amp.jvp(cj, tj).cpu().numpy()) < 1e-12, j
        refv = amp.vjp(cj, g[j])
        qv = lay.views(Q[j])
        _close_keys(qv, {kk: refv[kk].reshape(qv[kk].shape) for kk in keys}, j)


def test_amp2_large_B(ift, restore):
    """C5's 4096^2 grid (B = 1,197,363 bins, 1170 tiles: the carries over
    the tiles in several chunks)"""
    from nifty_amd import _native
    cf, amp, keys, c, (const, keep), lin, lay, D, off = _setup(ift, (4096, 4096), CF_ARGS, 4)
    assert _native.load().nft_amp2_tiles(amp.B, 4, 2) == 1170
    da = torch.empty((amp.B, 4), dtype=torch.float64, device=D.device)
    amp.native_jvp_batched(lin, D, off, da, interleave=True)
    g = torch.randn((4, amp.B), dtype=torch.float64, device=D.device)
    Q = torch.zeros_like(D)
    amp.native_vjp_batched(lin, g, Q, off)
    for j in (0, 3):
        tj = {kk: lay.views(D[j])[kk] for kk in keys}
        assert rel(da[:, j].cpu().numpy(), amp.jvp(c, tj).cpu().numpy()) < 1e-12
        refv = amp.vjp(c, g[j])
        qv = lay.views(Q[j])
        _close_keys(qv, {kk: refv[kk].reshape(qv[kk].shape) for kk in keys}, j)


@pytest.mark.parametrize("iters", [8, 25])
def test_carried_amplitude_cg(ift, iters):
    """The sampling CG with the amplitude keys' direction / update / finalize
    carried by the two-phase kernels (default) against the separate
    direction, update and finalize launches: the same iterates to rounding;
    single == batched bitwise on the carried path"""
    from nifty_amd.minimization import fused_cg
    cf, lh, pos = _los_problem(ift, golden("losmetric64.npz"))
    dtype, f_lh = lh.get_transformation()
    fl = f_lh(ift.Linearization.make_var(pos))
    A = (ift.SandwichOperator.make(fl.jac, ift.ScalingOperator(f_lh.target, 1., dtype))
         + ift.ScalingOperator(fl.domain, 1., float))
    core, W, shift = fused_cg.fusable_metric(A)
    assert core.amp2_tiles(3) > 0 and core.amp2_tiles(1) > 0
    ic = ift.GradientNormController(iteration_limit=iters)
    with ift.random.Context(11):   # independent of the tests before it
        es = [ift.QuadraticEnergy(0.1 * ift.from_random(cf.domain, "normal"), A,
                                  ift.from_random(cf.domain, "normal")) for _ in range(3)]
    out = {}
    for on in (True, False):
        fused_cg._AMP2 = on
        try:
            out[on] = [r for r in fused_cg.FusedCGBatch(core, W, shift, [copy.deepcopy(ic) for _ in es]).run(es)]
            if on:
                single = [fused_cg.FusedCG(core, W, shift, copy.deepcopy(ic)).run(e) for e in es]
        finally:
            fused_cg._AMP2 = True
    for j in range(3):
        assert out[True][j][1] == out[False][j][1] == single[j][1]
        for key in cf.domain.keys():
            a = out[True][j][0].position[key].val
            assert torch.equal(a, single[j][0].position[key].val), key
            if iters <= 8:
                assert rel(a.cpu().numpy(), out[False][j][0].position[key].val.cpu().numpy()) < 1e-11, key
        # past ~10 steps the rounding differences grow ~10x per step (the
        # reference's own backends diverge alike): whole vectors, looser
        x1 = np.concatenate([out[True][j][0].position[k].val.cpu().numpy().ravel() for k in cf.domain.keys()])
        x2 = np.concatenate([out[False][j][0].position[k].val.cpu().numpy().ravel() for k in cf.domain.keys()])
        assert rel(x1, x2) < (1e-11 if iters <= 8 else 5e-4)
        # the residuals as whole vectors (a scalar key's residual is a small
        # difference of large terms)
        g1 = np.concatenate([out[True][j][0].gradient[k].val.cpu().numpy().ravel() for k in cf.domain.keys()])
        g2 = np.concatenate([out[False][j][0].gradient[k].val.cpu().numpy().ravel() for k in cf.domain.keys()])
        if iters <= 8:
            assert rel(g1, g2) < 1e-9
        else:   # the small late residual carries the grown rounding differences
            # (its norm varies by tens of percent between summation orders):
            # the energy, stationary at the solution, is the stable measure
            # (seed-dependent: 1e-7 .. 1.1e-6 relative over the seeds tried)
            e1, e2 = out[True][j][0].value, out[False][j][0].value
            assert abs(e1 - e2) <= 5e-6 * abs(e2), (e1, e2)


def test_logging_controller_sees_every_energy(ift):
    """A count-only controller with an energy history (enable_logging) is not
    silent: every check reads the energy, so the CG runs unchunked; the
    iterates equal the silent controller's to rounding and the history holds the
    start energy (twice, as the reference's start + first check record it) and
    one energy per check, the last one the final energy's value"""
    from nifty_amd.minimization import fused_cg
    cf, lh, pos = _los_problem(ift, golden("losmetric64.npz"))
    dtype, f_lh = lh.get_transformation()
    fl = f_lh(ift.Linearization.make_var(pos))
    A = (ift.SandwichOperator.make(fl.jac, ift.ScalingOperator(f_lh.target, 1., dtype))
         + ift.ScalingOperator(fl.domain, 1., float))
    core, W, shift = fused_cg.fusable_metric(A)
    e = ift.QuadraticEnergy(0.1 * ift.from_random(cf.domain, "normal"), A, ift.from_random(cf.domain, "normal"))
    silent = ift.GradientNormController(iteration_limit=8)
    logged = ift.GradientNormController(iteration_limit=8)
    logged.enable_logging()
    assert fused_cg._count_silent(silent) and not fused_cg._count_silent(logged)
    r0 = fused_cg.FusedCG(core, W, shift, silent).run(e)
    r1 = fused_cg.FusedCG(core, W, shift, logged).run(e)
    # reading the value streams b and leaves the carried iteration: the same
    # iterates to rounding
    x0 = np.concatenate([r0[0].position[k].val.cpu().numpy().ravel() for k in cf.domain.keys()])
    x1 = np.concatenate([r1[0].position[k].val.cpu().numpy().ravel() for k in cf.domain.keys()])
    assert rel(x1, x0) < 1e-10
    h = logged.history
    # start() logs and then checks (itcount -1 -> 0), both record the start
    # energy (iteration_controllers.py:95-112): 2 + 8 checks
    assert len(h.energy_values) == logged._itcount + 2 == 10
    assert h.energy_values[0] == h.energy_values[1]
    assert h.energy_values[-1] == pytest.approx(r1[0].value, rel=1e-9)


def test_amp2_calls_on_two_streams(ift, restore):
    """Calls of the two-phase kernels (device-global arrival counters, one
    shared workspace) issued alternately on two streams with no host sync
    between them run one after the other (nft_amp2's stream guard): bitwise
    the results of the same calls on one stream."""
    _toggle(1)
    with ift.random.Context(31):
        cf, amp, keys, c, (const, keep), lin, lay, D, off = _setup(ift, (2048, 2048), CF_ARGS, 4)
    B, dev = amp.B, D.device
    gen = torch.Generator(device=dev).manual_seed(31)
    gs = [torch.randn((4, B), dtype=torch.float64, device=dev, generator=gen) for _ in range(6)]
    Ds = [D * (1.0 + 0.125 * i) for i in range(6)]

    def run(i):
        da = torch.empty((B, 4), dtype=torch.float64, device=dev)
        amp.native_jvp_batched(lin, Ds[i], off, da, interleave=True)
        Q = torch.zeros_like(D)
        amp.native_vjp_batched(lin, gs[i], Q, off, Ds[i], 0.75)
        return da, Q
    ref = [run(i) for i in range(6)]
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    cur = torch.cuda.current_stream()
    s1.wait_stream(cur)
    s2.wait_stream(cur)
    out = []
    for i in range(6):
        with torch.cuda.stream(s1 if i % 2 == 0 else s2):
            out.append(run(i))
    torch.cuda.synchronize()
    for i in range(6):
        assert torch.equal(out[i][0], ref[i][0]), i
        assert torch.equal(out[i][1], ref[i][1]), i


def test_two_captured_iteration_graphs_bitwise(ift):
    """Two HIP graphs of the bench's batched CG iteration (bench.cg_iteration:
    the carried iteration with the two-phase amplitude kernels, whose arrival
    counters and workspace every launch shares) on two buffer sets, replayed
    back to back A B A B: bitwise the same four iterations run eagerly."""
    import bench
    from nifty_amd import _native
    from nifty_amd.minimization import fused_cg
    cf, R, lh, pos, _ = bench.build_problem(ift, 256, 2048, "C3")
    lib = _native.load()
    k = 4
    core, W, shift, XS = bench.probe_setup(ift, lh, pos, k)
    n = XS.shape[1]

    def fresh(scale):
        X, Rr, D = (XS[i * k:(i + 1) * k] * scale for i in range(3))
        SC = torch.zeros((k, _native.CG_NSCALARS), dtype=torch.float64, device=XS.device)
        SC[:, _native.CG_GAMMA] = 1.0
        SC[:, _native.CG_GPREV] = 1.0
        ws = torch.empty(k * lib.nft_reduce_workspace(n), dtype=torch.uint8, device=XS.device)
        return (X.clone(), Rr.clone(), D.clone(), torch.zeros_like(X), SC, ws)

    warm = fresh(1.0)
    bench.cg_iteration(lib, core, W, shift, warm, k)   # plans, tables, first-use allocations
    torch.cuda.synchronize()
    eager = {"A": fresh(1.0), "B": fresh(0.5)}
    for name in "ABAB":
        bench.cg_iteration(lib, core, W, shift, eager[name], k)
    graph = {"A": fresh(1.0), "B": fresh(0.5)}
    gr = {name: fused_cg._capture(lambda b=graph[name]: bench.cg_iteration(lib, core, W, shift, b, k))
          for name in "AB"}
    for name in "ABAB":
        gr[name].replay()
    torch.cuda.synchronize()
    for name in "AB":
        for i, (a, b) in enumerate(zip(eager[name][:5], graph[name][:5])):
            assert torch.equal(a, b), (name, i)

