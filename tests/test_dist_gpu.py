"""Sharded draw_samples + SampledKLEnergy end to end on the GPU, 2 ranks.

Two freshly spawned processes share cuda:0 and a gloo process group (the box
has one GPU; on an 8-GPU node the same code runs one process per GPU over
RCCL).  As the reference's test_mpi/test_kl.py:46-114 demands, the KL value
and gradient in deterministic mode (the pairwise tree over point-to-point
messages, utilities._tree_sum) are bit-identical to the 1-rank run, and the
MGVI samples come in mirrored pairs (test_mpi/test_kl.py:117-133).  Fast mode
(one all-reduce) agrees to rounding.  The problem is losmetric64's
(sigmoid o LOS, 64^2); 2 mirrored pairs, so both ranks hold >= 2 samples and
run the batched KL pass like the 1-rank run."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CF_ARGS = dict(offset_mean=0, offset_std=(1e-3, 1e-6), fluctuations=(1., 0.8),
               loglogavgslope=(-3., 1), flexibility=(2, 1.), asperity=(0.5, 0.4))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(comm):
    """{mode: (kl value, gradient dict, local samples)} for MGVI and geoVI,
    deterministic and fast reductions"""
    import nifty_amd as ift
    from nifty_amd import utilities
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from conftest import golden
    G = golden("losmetric64.npz")
    sp = ift.RGSpace((64, 64))
    cf = ift.SimpleCorrelatedField(sp, **CF_ARGS)
    R = ift.LOSResponse(sp, starts=list(G["starts"]), ends=list(G["ends"]))
    N = ift.ScalingOperator(R.target, 1e-3, np.float64)
    lh = ift.GaussianEnergy(ift.makeField(R.target, G["data"]), inverse_covariance=N.inverse) @ R(ift.sigmoid(cf))
    pos = ift.MultiField.from_dict({k: ift.makeField(cf.domain[k], G["pos_" + k]) for k in cf.domain.keys()},
                                   cf.domain)
    H = ift.StandardHamiltonian(lh, ift.GradientNormController(iteration_limit=10))
    out = {}
    for geo in (False, True):
        for det in (True, False):
            utilities.DETERMINISTIC_ALLREDUCE = det
            mini = ift.NewtonCG(ift.GradientNormController(iteration_limit=1)) if geo else None
            ift.random.push_sseq_from_seed(51)
            kl = ift.SampledKLEnergy(pos, H, 2, mini, True, comm=comm)
            ift.random.pop_sseq()
            # the KL metric (kl_energies.py:340-350): batched per-sample
            # metrics, one reduction per application
            with ift.random.Context(7):
                v = ift.from_random(cf.domain, "normal")
            mvf = kl.apply_metric(v)
            mv = {k: mvf[k].val.cpu().numpy() for k in mvf.keys()}
            utilities.DETERMINISTIC_ALLREDUCE = False
            grad = {k: kl.gradient[k].val.cpu().numpy() for k in kl.gradient.keys()}
            sl = kl.samples
            loc = [{k: sl._r[i][k].val.cpu().numpy() for k in cf.domain.keys()} for i in range(len(sl._r))]
            out[(geo, det)] = (kl.value, grad, loc, list(sl._n), sl.n_samples, mv)
    return out


def _worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world), LOCAL_RANK=str(rank), HSA_ENABLE_IPC_MODE_LEGACY="0")
        sys.path.insert(0, ROOT)
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import nifty_amd as ift
        ift.config.set_device("cuda:0")
        res = _run(ift.TorchComm())
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, res))
    except Exception as e:  # surface the failure in the parent
        import traceback
        q.put((rank, "ERROR " + repr(e) + "\n" + traceback.format_exc()))


@pytest.fixture(scope="module")
def sharded(dev):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            r, res = q.get(timeout=180)
            out[r] = res
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r, res in out.items():
        assert not isinstance(res, str), res
    return out


@pytest.fixture(scope="module")
def single(dev):
    import nifty_amd as ift
    ift.config.set_device("cuda:0")
    return _run(None)


@pytest.mark.parametrize("geo", [False, True])
def test_sharded_kl_bitwise_deterministic(sharded, single, geo):
    v1, g1, loc1, neg1, n1 = single[(geo, True)][:5]
    for r in sharded:
        v, g, loc, neg, n = sharded[r][(geo, True)][:5]
        assert n == n1 == 4
        assert v == v1, (r, v, v1)
        for k in g1:
            np.testing.assert_array_equal(g[k], g1[k], err_msg=f"rank {r} key {k}")
    # the ranks' local samples are the 1-rank run's, in order
    both = sharded[0][(geo, True)][2] + sharded[1][(geo, True)][2]
    assert len(both) == len(loc1) == 4
    for a, b in zip(both, loc1):
        for k in b:
            np.testing.assert_array_equal(a[k], b[k])


@pytest.mark.parametrize("geo", [False, True])
def test_sharded_kl_fast_mode(sharded, single, geo):
    v1, g1 = single[(geo, False)][:2]
    for r in sharded:
        v, g = sharded[r][(geo, False)][:2]
        assert abs(v - v1) <= 1e-13 * abs(v1)
        for k in g1:
            np.testing.assert_allclose(g[k], g1[k], rtol=1e-12, atol=1e-14 * np.abs(g1[k]).max())
    assert sharded[0][(geo, False)][0] == sharded[1][(geo, False)][0]


def test_sharded_mgvi_mirrored(sharded):
    """MGVI residuals of a pair are one residual with neg flags (False, True),
    the pair held by one rank (test_mpi/test_kl.py:117-133)"""
    for r in sharded:
        _, _, loc, neg = sharded[r][(False, True)][:4]
        assert neg == [False, True]
        for k in loc[0]:
            np.testing.assert_array_equal(loc[0][k], loc[1][k])


@pytest.mark.parametrize("geo", [False, True])
def test_sharded_kl_metric(sharded, single, geo):
    """KL metric application on 2 ranks: bit-identical to 1 rank in
    deterministic mode, to rounding with the one all-reduce"""
    m1 = single[(geo, True)][5]
    for r in sharded:
        m = sharded[r][(geo, True)][5]
        for k in m1:
            np.testing.assert_array_equal(m[k], m1[k], err_msg=f"rank {r} key {k}")
    m1 = single[(geo, False)][5]
    for r in sharded:
        m = sharded[r][(geo, False)][5]
        for k in m1:
            np.testing.assert_allclose(m[k], m1[k], rtol=1e-12, atol=1e-14 * np.abs(m1[k]).max())
