"""Sharded draw_samples + SampledKLEnergy + KL metric at world sizes 3 and 8
(gloo process groups, every rank on cuda:0 of the one-GPU box; on an 8-GPU
node the same code runs one process per GPU over RCCL).

As the reference's test_mpi/test_kl.py:46-114 demands, the KL value, its
gradient and the KL metric applied to a vector are bit-identical to the
1-rank run in deterministic mode (the reference's pairwise tree over
point-to-point messages, utilities._tree_sum), and every rank's local
samples are the 1-rank run's samples of its shareRange slice
(src/utilities.py:268-292, kl_energies.py:140-145):

  world 8, n_samples 16 mirrored: 2 pairs per rank (BASELINE C4's share)
  world 8, n_samples 32 mirrored: 4 pairs per rank (BASELINE C5's share)
  world 3, n_samples 4 mirrored:  8 samples as 3 + 3 + 2 -- rank 0 ends on
                                  the first half of a pair, rank 1 starts on
                                  its second half (a split mirrored pair,
                                  which re-draws y from the same seed)

geoVI (NewtonCG, one step) on the losmetric64 problem (sigmoid o LOS, 64^2);
MGVI as well at world 3."""
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
CASES = {8: [(16, True), (32, True)], 3: [(4, True), (4, False)]}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(comm, cases):
    """{(n_samples, geo): (kl value, gradient, local samples, neg flags,
    n_samples, KL metric applied to a fixed vector)} in deterministic mode"""
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
    H = ift.StandardHamiltonian(lh, ift.GradientNormController(iteration_limit=8))
    out = {}
    for nsamp, geo in cases:
        utilities.DETERMINISTIC_ALLREDUCE = True
        try:
            mini = ift.NewtonCG(ift.GradientNormController(iteration_limit=1)) if geo else None
            ift.random.push_sseq_from_seed(61)
            kl = ift.SampledKLEnergy(pos, H, nsamp, mini, True, comm=comm)
            ift.random.pop_sseq()
            with ift.random.Context(7):
                v = ift.from_random(cf.domain, "normal")
            mvf = kl.apply_metric(v)
            mv = {k: mvf[k].val.cpu().numpy() for k in mvf.keys()}
            grad = {k: kl.gradient[k].val.cpu().numpy() for k in kl.gradient.keys()}
            value = kl.value
        finally:
            utilities.DETERMINISTIC_ALLREDUCE = False
        sl = kl.samples
        loc = [{k: sl._r[i][k].val.cpu().numpy() for k in cf.domain.keys()} for i in range(len(sl._r))]
        out[(nsamp, geo)] = (value, grad, loc, list(sl._n), sl.n_samples, mv)
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
        res = _run(ift.TorchComm(), CASES[world])
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, res))
    except Exception as e:  # surface the failure in the parent
        import traceback
        q.put((rank, "ERROR " + repr(e) + "\n" + traceback.format_exc()))


def _spawn(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            r, res = q.get(timeout=300)
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
    return _run(None, sorted({c for cs in CASES.values() for c in cs}))


@pytest.mark.parametrize("world", [3, 8])
def test_sharded_bitwise_vs_one_rank(single, world):
    from nifty_amd import utilities
    sharded = _spawn(world)
    for case in CASES[world]:
        nsamp, geo = case
        v1, g1, loc1, neg1, n1, m1 = single[case]
        total = 2 * nsamp
        assert n1 == total and len(loc1) == total
        gathered = []
        for r in range(world):
            v, g, loc, neg, n, m = sharded[r][case]
            assert n == total
            assert v == v1, (world, case, r, v, v1)
            for k in g1:
                np.testing.assert_array_equal(g[k], g1[k], err_msg=f"{world} {case} rank {r} grad {k}")
            for k in m1:
                np.testing.assert_array_equal(m[k], m1[k], err_msg=f"{world} {case} rank {r} metric {k}")
            lo, hi = utilities.shareRange(total, world, r)
            assert len(loc) == hi - lo, (r, len(loc), lo, hi)
            assert neg == neg1[lo:hi]
            gathered += loc
        for i, (a, b) in enumerate(zip(gathered, loc1)):
            for k in b:
                np.testing.assert_array_equal(a[k], b[k], err_msg=f"{world} {case} sample {i} key {k}")
    if world == 3:
        # the split pair: rank 0 ends on the first half of pair 1, rank 1 starts
        # on its second half
        assert utilities.shareRange(8, 3, 0) == (0, 3) and utilities.shareRange(8, 3, 1) == (3, 6)
