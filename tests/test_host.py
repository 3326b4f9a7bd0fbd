"""CPU: the C-ABI library loads and exports every symbol of include/nifty_amd.h,
and the host-side logic of the package (geometry, binning, RNG streams,
sharding, controllers, LOS construction, operator algebra bookkeeping)
matches the reference's golden vectors.  No GPU compute here."""
import os
import re

import numpy as np
import pytest

from conftest import ROOT, golden


def _header_symbols():
    txt = open(os.path.join(ROOT, "include", "nifty_amd.h")).read()
    return sorted(set(re.findall(r"^\s*(?:const char\*|void|int|int64_t|size_t)\s+(nft_\w+)\s*\(", txt, re.M)))


def test_library_exports_every_header_symbol():
    import ctypes
    from nifty_amd import _native
    assert os.path.exists(_native.LIB_PATH), "run __graft_entry__.build() first"
    lib = ctypes.CDLL(_native.LIB_PATH)
    syms = _header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(lib, s), s
    # the Python binding covers exactly the header
    assert sorted(_native.SIGNATURES) == syms
    _native.load()


def test_folded_prologue_block_count():
    """nft_hartley_dir_blocks (pure host arithmetic): 2-D / 3-D grids with
    n_last/2+1 <= 2560 take the row-staged prologue, one block per group of
    mirror rows (prod over the leading axes of n/2+1); 1-D and longer rows
    the cell grid prod(n/2+1), last axis padded to 64, 256 cells per block"""
    from nifty_amd import _native
    assert _native.hartley_dir_blocks((2048, 2048)) == 1025
    assert _native.hartley_dir_blocks((64, 30)) == 33
    assert _native.hartley_dir_blocks((8, 8, 130)) == 5 * 5
    assert _native.hartley_dir_blocks((512, 512, 512)) == 257 * 257
    assert _native.hartley_dir_blocks((4, 8192)) == (3 * 4160 + 255) // 256
    assert _native.hartley_dir_blocks((100,)) == 1
    assert _native.hartley_dir_blocks((0, 4)) == 0


def test_no_cpu_fallback():
    import torch
    from nifty_amd import _native
    with pytest.raises(_native.NativeError):
        _native.hartley(torch.zeros(8, dtype=torch.float64), (0,))
    with pytest.raises(_native.NativeError):
        _native.dot(torch.zeros(8, dtype=torch.float64), torch.zeros(8, dtype=torch.float64))


def test_powerspace_bit_exact():
    import nifty_amd as ift
    G = golden("geometry.npz")
    for i in range(int(G["nspaces"])):
        shape = tuple(int(s) for s in G[f"s{i}_shape"])
        h = ift.RGSpace(shape, distances=tuple(G[f"s{i}_pos_dist"]))
        h = h.get_default_codomain()
        assert np.allclose(h.distances, G[f"s{i}_dist"], rtol=1e-15, atol=0)
        ps = ift.PowerSpace(h)
        np.testing.assert_array_equal(ps.pindex, G[f"s{i}_pindex"])
        np.testing.assert_array_equal(ps.k_lengths, G[f"s{i}_k_lengths"])
        np.testing.assert_array_equal(ps.dvol, G[f"s{i}_dvol"])
        np.testing.assert_array_equal(h.get_unique_k_lengths(), G[f"s{i}_uniq"])


def test_bin_index_matches_bincount_order():
    from nifty_amd.operators.distributors import BinIndex
    G = golden("geometry.npz")
    p = G["s1_pindex"]
    b = BinIndex(p, int(p.max()) + 1, "cpu")
    perm = b.perm.numpy()
    offs = b.offsets.numpy()
    for bin_ in (0, 1, 5, int(p.max())):
        members = perm[offs[bin_]:offs[bin_ + 1]]
        assert np.all(np.diff(members) > 0)          # ascending pixel order = bincount order
        assert np.all(p.ravel()[members] == bin_)


def test_bin_fold_layout_host():
    """Host half of the mirror-folded Jacobian bin sums: BinIndex(fold=True)
    indexes the fundamental cell; summing each cell point's mirror images
    (numpy restatement of nft_bin_fold) and then the cell's bins reproduces
    np.bincount on the full grid to rounding.  Asymmetric grids do not fold."""
    import nifty_amd as ift
    from nifty_amd.operators.distributors import BinIndex
    rng = np.random.default_rng(2)
    for shape in [(64, 64), (63, 67), (16, 18, 20), (4097,)]:
        grid = np.asarray(ift.PowerSpace(ift.RGSpace(shape, harmonic=True)).pindex)
        nb = int(grid.max()) + 1
        f = BinIndex(grid, nb, "cpu", fold=True).fold
        assert f is not None and f["nf"] == int(np.prod([n // 2 + 1 for n in shape]))
        x = rng.standard_normal(shape)
        xf = x
        for ax, n in enumerate(shape):
            q = np.arange(n // 2 + 1)
            two = ((q != 0) & (2 * q != n)).reshape([-1 if a == ax else 1 for a in range(len(shape))])
            xf = np.take(xf, q, axis=ax) + np.where(two, np.take(xf, (n - q) % n, axis=ax), 0.)
        xf = xf.ravel()
        perm, offs = f["perm"].numpy(), f["offsets"].numpy()
        got = np.array([xf[perm[offs[i]:offs[i + 1]]].sum() for i in range(nb)])
        g = grid.ravel()
        ref = np.bincount(g, weights=x.ravel(), minlength=nb)
        bound = 1e-15 * np.bincount(g, minlength=nb) * np.bincount(g, weights=np.abs(x).ravel(), minlength=nb)
        assert np.all(np.abs(got - ref) <= bound), shape
    assert BinIndex(rng.integers(0, 50, (64, 64)), 50, "cpu", fold=True).fold is None


def test_random_streams_match_reference():
    import nifty_amd as ift
    G = golden("random.npz")
    dom = ift.makeDomain({"zeta": ift.RGSpace(5), "alpha": ift.RGSpace((2, 3)),
                          "mid": ift.DomainTuple.scalar_domain()})
    with ift.random.Context(7):
        mf = ift.from_random(dom, "normal", std=2.)
    for k in ("alpha", "mid", "zeta"):
        np.testing.assert_array_equal(np.asarray(mf[k]), G["mf_" + k])
    ift.random.push_sseq_from_seed(27)
    ss = ift.random.spawn_sseq(3)
    for i, s in enumerate(ss):
        with ift.random.Context(s):
            np.testing.assert_array_equal(ift.random.current_rng().standard_normal(4), G[f"child{i}"])
    ift.random.pop_sseq()


@pytest.mark.parametrize("nwork,nshares", [(8, 1), (8, 2), (8, 3), (4, 8), (16, 8), (2, 2)])
def test_share_range_partition(nwork, nshares):
    from nifty_amd.utilities import shareRange
    got = [shareRange(nwork, nshares, r) for r in range(nshares)]
    assert got[0][0] == 0 and got[-1][1] == nwork
    for (a, b), (c, d) in zip(got[:-1], got[1:]):
        assert b == c
    sizes = [b - a for a, b in got]
    assert max(sizes) - min(sizes) <= 1


def test_los_construction_bit_exact():
    from nifty_amd.library.los_response import los_coo
    G = golden("los.npz")
    for i in range(3):
        shape = tuple(int(s) for s in G[f"l{i}_shape"])
        dist = tuple(1. / np.array(shape))
        rows, cols, w, nlos = los_coo(shape, dist, G[f"l{i}_starts"], G[f"l{i}_ends"])
        np.testing.assert_array_equal(rows, G[f"l{i}_row"])
        np.testing.assert_array_equal(cols, G[f"l{i}_col"])
        np.testing.assert_array_equal(w, G[f"l{i}_wgt"])


@pytest.mark.parametrize("i", range(3))
def test_los_box_plan_layout(i):
    """The box-blocked layout the nft_los kernels consume reproduces the
    reference's COO matvec / rmatvec (golden COO + vectors, los.npz), via a
    numpy restatement of the kernels' arithmetic; plus a forced split of
    over-full boxes into several work items."""
    import scipy.sparse
    from nifty_amd.library import los_response as lr
    G = golden("los.npz")
    shape = tuple(int(s) for s in G[f"l{i}_shape"])
    rows, cols, w = G[f"l{i}_row"], G[f"l{i}_col"], G[f"l{i}_wgt"]
    nlos = len(G[f"l{i}_y"])
    P = lr.box_plan(rows, cols, w, shape, nlos)
    assert P["item_seg"][-1] == P["nseg"] and P["box_ent"][-1] == len(rows)
    assert np.all(np.diff(P["item_seg"]) <= lr.BOX)
    assert np.all(P["seg_ent"][P["item_seg"][1:]] - P["seg_ent"][P["item_seg"][:-1]] <= lr.LOS_CAP_F)
    x, y = G[f"l{i}_x"], G[f"l{i}_y"]
    assert np.allclose(lr.box_plan_apply(P, x, "times"), G[f"l{i}_Rx"], rtol=1e-13, atol=0)
    assert np.allclose(lr.box_plan_apply(P, y, "adjoint"), G[f"l{i}_Rty"].ravel(), rtol=1e-13, atol=1e-300)
    old = lr.LOS_CAP_F
    try:
        lr.LOS_CAP_F = 40
        P2 = lr.box_plan(rows, cols, w, shape, nlos)
        assert P2["nitems"] > P["nitems"]
        assert np.allclose(lr.box_plan_apply(P2, x, "times"), G[f"l{i}_Rx"], rtol=1e-13, atol=0)
    finally:
        lr.LOS_CAP_F = old
    del scipy


def test_controllers_semantics():
    import nifty_amd as ift

    class E:
        def __init__(self, v, g):
            self.value, self.gradient_norm = v, g

    c = ift.AbsDeltaEnergyController(deltaE=0.5, convergence_level=2, iteration_limit=10)
    assert c.start(E(10., 1.)) == c.CONTINUE
    assert c.check(E(9.8, 1.)) == c.CONTINUE      # ccount 1
    assert c.check(E(9.7, 1.)) == c.CONVERGED     # ccount 2
    c = ift.GradientNormController(iteration_limit=3)
    assert c.start(E(0, 1.)) == c.CONTINUE
    assert c.check(E(0, 1.)) == c.CONTINUE
    assert c.check(E(0, 1.)) == c.CONTINUE
    assert c.check(E(0, 1.)) == c.CONVERGED
    c = ift.GradientNormController(tol_abs_gradnorm=0.1)
    assert c.start(E(0, 1.)) == c.CONTINUE
    assert c.check(E(0, 0.01)) == c.CONVERGED


def test_operator_algebra_bookkeeping_cpu():
    """Chain/sum simplification of scalars and domains (chain_operator.py:54-110,
    sum_operator.py:64-200) runs on host-side objects only."""
    import nifty_amd as ift
    sp = ift.RGSpace(8)
    s2 = ift.ScalingOperator(sp, 2.)
    s3 = ift.ScalingOperator(sp, 3.)
    op = s2 @ s3
    assert isinstance(op, ift.ScalingOperator) and op._factor == 6.
    op = s2 + s3
    assert isinstance(op, ift.ScalingOperator) and op._factor == 5.
    assert op.adjoint._factor == 5.
    assert op.inverse._factor == 0.2
    gr = ift.GeometryRemover(sp)
    ch = gr @ s2
    assert isinstance(ch, ift.ChainOperator)
    assert ch.target == ift.DomainTuple.make(ift.UnstructuredDomain(8))
    x = ift.full(sp, 1.)
    assert np.allclose(np.asarray(ch(x)), 2.)
    with pytest.raises(NotImplementedError):
        ift.HarmonicTransformOperator(sp.get_default_codomain()).inverse
        ift.HarmonicTransformOperator(sp.get_default_codomain()).inverse_times(x)


def test_cf_latent_domain_matches_reference_keys():
    import nifty_amd as ift
    G = golden("cf128.npz")
    sp = ift.RGSpace((128, 128))
    cf = ift.SimpleCorrelatedField(sp, offset_mean=0, offset_std=(1e-3, 1e-6), fluctuations=(1., 0.8),
                                   loglogavgslope=(-3., 1), flexibility=(2, 1.), asperity=(0.5, 0.4))
    keys = sorted(k[2:] for k in G.files if k.startswith("x_"))
    assert list(cf.domain.keys()) == keys
    for k in keys:
        assert cf.domain[k].shape == G["x_" + k].shape


def test_cf_amplitude_cpu_matches_golden():
    """B-sized amplitude math (no grid work) evaluated on host tensors."""
    import nifty_amd as ift
    import torch
    G = golden("cf128.npz")
    sp = ift.RGSpace((128, 128))
    cf = ift.SimpleCorrelatedField(sp, offset_mean=0, offset_std=(1e-3, 1e-6), fluctuations=(1., 0.8),
                                   loglogavgslope=(-3., 1), flexibility=(2, 1.), asperity=(0.5, 0.4))
    lat = {k: torch.from_numpy(np.array(G["x_" + k])) for k in cf.amplitude.domain.keys()}
    a, c = cf.amp.forward(lat)
    assert np.max(np.abs(a.numpy() - G["amp"])) <= 1e-14 * np.max(np.abs(G["amp"]))


def test_rng_prefetch_bit_identical():
    """Prefetched draws (random.prefetch) equal direct draws; a request that
    leaves the recorded script rebuilds the exact generator state."""
    from nifty_amd import random as R
    R.push_sseq_from_seed(123)
    try:
        kids = R.predict_spawn(3)
        ref = []
        spawned = R.spawn_sseq(3)
        assert [k.spawn_key for k in kids] == [k.spawn_key for k in spawned]
        for ss in spawned:
            with R.Context(ss):
                a = R.Random.normal(np.float64, (50, 7))
                b = R.Random.uniform(np.float64, (5,))
                c = R.Random.normal(np.float64, (3,))
            ref.append((a, b, c))
        script = [("normal", (0.0, 1.0, (50, 7)), ()), ("uniform", (0.0, 1.0, (5,)), ())]
        # same seeds again: spawn from a fresh parent with the same entropy
        R.pop_sseq()
        R.push_sseq_from_seed(123)
        nxt = R.predict_spawn(3)
        R.prefetch(nxt, script)
        out = []
        for ss in R.spawn_sseq(3):
            ctx = R.Context(ss)
            with ctx:
                a = R.Random.normal(np.float64, (50, 7))
                b = R.Random.uniform(np.float64, (5,))
                c = R.Random.normal(np.float64, (3,))   # beyond the script: generator rebuilt
            out.append((a, b, c))
            assert ctx.script[0][0] == "normal"
        for (a, b, c), (x, y, z) in zip(ref, out):
            np.testing.assert_array_equal(a, x)
            np.testing.assert_array_equal(b, y)
            np.testing.assert_array_equal(c, z)
        # mismatching first request: falls back to the generator
        R.prefetch(R.predict_spawn(1), script)
        ss = R.spawn_sseq(1)[0]
        with R.Context(ss):
            u = R.Random.uniform(np.float64, (4,))
        np.testing.assert_array_equal(u, np.random.default_rng(ss).uniform(0., 1., (4,)))
    finally:
        R.pop_sseq()


def test_stat_calculator():
    """probing.StatCalculator (probing.py:24-71): Welford mean / unbiased var."""
    from nifty_amd.probing import StatCalculator
    rng = np.random.default_rng(3)
    xs = rng.normal(size=(7, 5))
    sc = StatCalculator()
    for x in xs:
        sc.add(x)
    np.testing.assert_allclose(sc.mean, xs.mean(0), rtol=1e-14)
    np.testing.assert_allclose(sc.var, xs.var(0, ddof=1), rtol=1e-13)


def test_checkpoint_roundtrip_cpu(tmp_path):
    """optimize_kl's data-only checkpoint files (minimization/checkpoint.py):
    fields / sample lists round-trip bit for bit with their domains rebuilt,
    the random state restores the exact stream (the reference pickles
    (sseq stack, generator stack), src/random.py:89-111), stale-free
    numbering is enforced."""
    import nifty_amd as ift
    from nifty_amd.minimization import checkpoint
    dom = ift.makeDomain({"a": ift.RGSpace((4, 6), distances=(0.5, 2.), harmonic=True),
                          "b": ift.UnstructuredDomain(3)})
    with ift.random.Context(4):
        m = ift.from_random(dom, "normal")
        r0 = ift.from_random(dom, "normal")
    sl = ift.ResidualSampleList(m, [r0, r0], [False, True])
    base = str(tmp_path / "last")
    sl.save(base)
    back = ift.ResidualSampleList.load(base)
    assert back.domain == dom and back.n_samples == 2 and list(back._n) == [False, True]
    for i in range(2):
        for k in dom.keys():
            assert np.array_equal(np.asarray(back.local_item(i)[k]), np.asarray(sl.local_item(i)[k]))
    # load onto the caller's domain object
    assert ift.ResidualSampleList.load_mean(base, dom).domain is dom
    with pytest.raises(FileExistsError):
        sl.save(base)
    sl.save(base, overwrite=True)
    ift.SampleList([m]).save(str(tmp_path / "map"))
    assert np.array_equal(np.asarray(ift.SampleList.load(str(tmp_path / "map")).local_item(0)["a"]),
                          np.asarray(m["a"]))
    # random state: the stream continues identically after a save / restore
    ift.random.push_sseq_from_seed(9)
    ift.random.current_rng().normal(size=5)
    st = checkpoint.random_state()
    checkpoint.save_json(str(tmp_path / "rs.json"), st)
    a = ift.random.current_rng().normal(size=7)
    s1 = ift.random.spawn_sseq(2)
    ift.random.current_rng().normal(size=3)
    checkpoint.set_random_state(checkpoint.load_json(str(tmp_path / "rs.json")))
    assert np.array_equal(ift.random.current_rng().normal(size=7), a)
    s2 = ift.random.spawn_sseq(2)
    assert [s.spawn_key for s in s1] == [s.spawn_key for s in s2]
    ift.random.pop_sseq()


def test_abi_host_code_under_asan():
    """The C ABI's host code (argument validation, workspace sizing, plan
    arithmetic, error formatting) built with AddressSanitizer (host side
    only, -Xarch_host -fsanitize=address) and driven through every entry
    point whose work ends on the host (tests/asan/abi_host_driver.cpp)."""
    import shutil
    import subprocess
    if shutil.which("make") is None or not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("hipcc / make not available")
    d = os.path.join(ROOT, "tests", "asan")
    b = subprocess.run(["make", "-C", d, "-j8"], capture_output=True, text=True, timeout=900)
    assert b.returncode == 0, b.stderr[-2000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0")
    r = subprocess.run([os.path.join(d, "build", "abi_host_driver")], capture_output=True, text=True,
                       timeout=120, env=env)
    assert "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    assert r.returncode == 0 and "abi host checks: ok" in r.stdout, (r.stdout, r.stderr[-2000:])


def test_worth_compacting_host():
    """FusedCGBatch compaction policy (fused_cg._worth_compacting): only with
    fewer live rows than buffer rows, and only while some live controller
    allows at least a few more iterations."""
    import nifty_amd as ift
    from nifty_amd.minimization.fused_cg import _worth_compacting
    c = [ift.GradientNormController(iteration_limit=10) for _ in range(3)]
    for x in c:
        x._itcount = 5
    assert not _worth_compacting(c, [0, 1, 2], 3)
    assert _worth_compacting(c, [0, 2], 3)
    for x in c:
        x._itcount = 8
    assert not _worth_compacting(c, [0, 2], 3)          # 2 iterations left
    c[2] = ift.AbsDeltaEnergyController(0.1)            # no limit
    c[2]._itcount = 50
    assert _worth_compacting(c, [0, 2], 3)


def test_trace_labels_host(tmp_path):
    """tools/trace_labels.py: the periodic tail of a kernel trace is split
    into iterations, dispatches labelled as bench.py labels them (the two
    unpack passes by order), per-label means and the iteration span."""
    import json
    import subprocess
    import sys
    names = ["void nft::amp2::jvp2a_kernel<2>(x)", "void nft::fast::fast_kernel<double, 64, 256, 3, false, false>(a)",
             "void nft::los_fwd_items<double, 4>(p)", "void nft::fast::fast_kernel<double, 64, 256, 3, false, false>(a)"]
    rows, t = [], 0
    for it in range(5):
        for j, nm in enumerate(names):
            d = 1000 * (j + 1)
            rows.append((nm, t, t + d))
            t += d + 100
    f = tmp_path / "trace.csv"
    with open(f, "w") as fh:
        fh.write("Kernel_Name,Start_Timestamp,End_Timestamp\n")
        for nm, a, b in rows:
            fh.write(f"\"{nm}\",{a},{b}\n")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, os.path.join(root, "tools", "trace_labels.py"), str(f), "3"],
                         capture_output=True, text=True, check=True).stdout
    d = json.loads(out)
    assert d["dispatches_per_iteration"] == 4
    lab = d["labels"]
    assert lab["fft_unpack"]["avg_us"] == 2.0 and lab["fft_unpack+cg"]["avg_us"] == 4.0
    assert lab["amp_jvp2a+dir"]["avg_us"] == 1.0 and lab["los_fwd_items"]["avg_us"] == 3.0
    assert d["iteration_span_us"] == 10.3
