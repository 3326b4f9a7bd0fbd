"""optimize_kl (src/minimization/optimize_kl.py:51-412) on the GPU: the
global-iteration driver against the reference's own run (optkl32.npz: MGVI,
MAP and geoVI iterations on the 32^2 Gaussian problem), and checkpoint /
resume -- an interrupted and resumed run reproduces the uninterrupted run bit
for bit (sample lists, random state and energy history restored from the
data-only checkpoint files, in the reference's layout)."""
import os

import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu

CF_ARGS = dict(offset_mean=0, offset_std=(1e-3, 1e-6), fluctuations=(1., 0.8),
               loglogavgslope=(-3., 1), flexibility=(2, 1.), asperity=(0.5, 0.4))


def _rel(a, b):
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


def _problem(ift, G):
    sp = ift.RGSpace((32, 32))
    cf = ift.SimpleCorrelatedField(sp, **CF_ARGS)
    R = ift.GeometryRemover(sp)
    N = ift.ScalingOperator(R.target, 0.01, np.float64)
    lh = ift.GaussianEnergy(ift.makeField(R.target, G["data"]), inverse_covariance=N.inverse) @ (R @ cf)
    pos = ift.MultiField.from_dict({k: ift.makeField(lh.domain[k], G["pos_" + k]) for k in lh.domain.keys()},
                                   lh.domain)
    return lh, pos


def _run(ift, lh, pos, total, **kw):
    means = []

    def inspect(sl, i):
        # a MAP iteration's SampleList holds its one position on rank 0 only
        m = sl._m if hasattr(sl, "_m") else sl.average()
        means.append({k: m[k].val.cpu().numpy() for k in m.keys()})
    ift.random.push_sseq_from_seed(61)
    try:
        sl, mean = ift.optimize_kl(
            lh, total, lambda i: 0 if i == 1 else 1,
            ift.NewtonCG(ift.GradientNormController(iteration_limit=2)),
            ift.GradientNormController(iteration_limit=8),
            lambda i: ift.NewtonCG(ift.GradientNormController(iteration_limit=1)) if i == 2 else None,
            initial_position=pos, return_final_position=True, inspect_callback=inspect, **kw)
    finally:
        ift.random.pop_sseq()
    return means, sl, mean


@pytest.fixture(scope="module")
def ift(dev):
    import nifty_amd
    return nifty_amd


def test_optimize_kl_golden(ift):
    G = golden("optkl32.npz")
    lh, pos = _problem(ift, G)
    means, sl, mean = _run(ift, lh, pos, 3)
    assert len(means) == 3
    for i, m in enumerate(means):
        tol = max(10 * float(G[f"it{i}_sens"]), 1e-10)
        for k, v in m.items():
            assert _rel(v, G[f"it{i}_mean_" + k]) < tol, (i, k, _rel(v, G[f"it{i}_mean_" + k]), tol)
    tol = max(10 * float(G["it2_sens"]), 1e-10)
    for k in mean.keys():
        assert _rel(mean[k].val.cpu().numpy(), G["final_" + k]) < tol, k
    assert sl.n_samples == 2
    for i in range(2):
        s = sl.local_item(i)
        for k in s.keys():
            assert _rel(s[k].val.cpu().numpy(), G[f"s{i}_" + k]) < tol, (i, k)


@pytest.mark.parametrize("strategy", ["last", "all"])
def test_optimize_kl_resume_bitwise(ift, tmp_path, strategy):
    G = golden("optkl32.npz")
    lh, pos = _problem(ift, G)
    full, sl_f, mean_f = _run(ift, lh, pos, 3, output_directory=str(tmp_path / "a"), save_strategy=strategy)
    d = tmp_path / "b"
    _run(ift, lh, pos, 2, output_directory=str(d), save_strategy=strategy)
    stem = "last" if strategy == "last" else "iteration_1"
    # the reference's layout (optimize_kl.py:297-317, sample_list.py:510-517)
    assert (d / "last_finished_iteration").read_text() == "1"
    for f in (f"nifty_random_state_{stem}.json", f"energy_history_{stem}.json", f"{stem}.0.npz"):
        assert os.path.isfile(d / "pickle" / f), f
    # interrupted after iteration 1, a MAP iteration: its stem holds the one
    # SampleList file and no mean (no stale residual files of iteration 0)
    assert not os.path.isfile(d / "pickle" / f"{stem}.mean.npz")
    assert not os.path.isfile(d / "pickle" / f"{stem}.1.npz")
    if strategy == "all":
        for f in ("iteration_0.mean.npz", "iteration_0.0.npz", "iteration_0.1.npz"):
            assert os.path.isfile(d / "pickle" / f), f
    res, sl_r, mean_r = _run(ift, lh, pos, 3, output_directory=str(d), save_strategy=strategy, resume=True)
    assert len(res) == 1      # only iteration 2 ran
    for k in full[2]:
        np.testing.assert_array_equal(res[0][k], full[2][k], err_msg=k)
    for k in mean_f.keys():
        np.testing.assert_array_equal(mean_r[k].val.cpu().numpy(), mean_f[k].val.cpu().numpy(), err_msg=k)
    assert (d / "last_finished_iteration").read_text() == "2"
    # resuming a finished run returns the stored result without iterating
    again, sl_a, mean_a = _run(ift, lh, pos, 3, output_directory=str(d), save_strategy=strategy, resume=True)
    assert again == [] and sl_a.n_samples == 2
    for k in mean_f.keys():
        np.testing.assert_array_equal(mean_a[k].val.cpu().numpy(), mean_f[k].val.cpu().numpy(), err_msg=k)
