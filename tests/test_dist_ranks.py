"""CPU: the multi-process reductions at world sizes 3 and 8 (gloo), the rank
counts of the BASELINE configs (C4 / C5: 8 ranks with 2 and 4 mirrored pairs
each) and an odd count that splits a mirrored pair across ranks.  Per world
size: shareRange covers the mirrored sample list exactly once; the
deterministic all-reduce (the reference's global pairwise tree,
src/utilities.py:331-390) and the KL value / gradient mean of
ResidualSampleList._average_tuple (sample_list.py:327-341) are bit-identical
to the single-process result for every split; fast mode sends ONE collective
per KL mean and agrees to rounding; ranks holding no samples get the mean.
(test/test_mpi/test_kl.py:46-114 demands the bit equality.)  The GPU-side
draws at 3 and 8 ranks: tests/test_dist_ranks_gpu.py.  No GPU compute."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# world size -> mirrored pairs in the sample list
CASES = {3: 5, 8: 16}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _values(n_total):
    """per-sample MultiFields with awkward magnitudes (order-sensitive sums)"""
    import nifty_amd as ift
    dom = ift.makeDomain({"a": ift.RGSpace(5), "b": ift.DomainTuple.scalar_domain(),
                          "xi": ift.RGSpace((3, 4))})
    rng = np.random.default_rng(23)
    out = []
    for _ in range(n_total):
        d = {k: rng.standard_normal(dom[k].shape) * 10.0 ** rng.integers(-8, 8, dom[k].shape)
             for k in dom.keys()}
        out.append(ift.MultiField.from_dict({k: ift.makeField(dom[k], v) for k, v in d.items()}, dom))
    return dom, out


def _arr(f, dom):
    return {k: np.asarray(f[k]) for k in dom.keys()}


def _worker(rank, world, npairs, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world), LOCAL_RANK=str(rank), OMP_NUM_THREADS="1")
        sys.path.insert(0, ROOT)
        import torch
        torch.set_num_threads(1)
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import nifty_amd as ift
        from nifty_amd import utilities
        comm = ift.TorchComm()
        res = {}
        n_total = 2 * npairs
        lo, hi = utilities.shareRange(n_total, world, rank)
        res["range"] = (lo, hi)
        dom, vals = _values(n_total)
        mean = vals[0]
        # deterministic tree and fast all-reduce of this rank's share
        res["det"] = _arr(utilities.allreduce_sum(vals[lo:hi], comm, deterministic=True), dom)
        res["fast"] = _arr(utilities.allreduce_sum(vals[lo:hi], comm, deterministic=False), dom)
        # the KL mean over the mirrored list (sample i mirrored when i is odd)
        neg = [(i % 2) == 1 for i in range(lo, hi)]
        sl = ift.ResidualSampleList(mean, vals[lo:hi], neg, comm)
        assert sl.n_samples == n_total and sl.n_local_samples == hi - lo
        kl = lambda s: (float(np.asarray(s["b"])), s)  # noqa: E731
        for det in (True, False):
            utilities.DETERMINISTIC_ALLREDUCE = det
            calls = []
            orig = comm.allreduce_tensor_
            comm.allreduce_tensor_ = lambda t: (calls.append(t.numel()), orig(t))[1]
            v, g = sl._average_tuple(kl)
            comm.allreduce_tensor_ = orig
            res[f"kl{int(det)}"] = (v, _arr(g, dom), len(calls))
            res[f"avg{int(det)}"] = _arr(sl.average(), dom)
        utilities.DETERMINISTIC_ALLREDUCE = False
        # 3 samples, all on the lowest ranks: the others hold none
        lo3, hi3 = utilities.shareRange(3, world, rank)
        few = [mean + v for v in vals[lo3:hi3]]
        sl3 = ift.ResidualSampleList(mean, vals[lo3:hi3], [False] * (hi3 - lo3), comm)
        utilities.DETERMINISTIC_ALLREDUCE = True
        v3, g3 = sl3._average_tuple(kl, lambda: (0.0, 0 * mean))
        utilities.DETERMINISTIC_ALLREDUCE = False
        res["few"] = (len(few), v3, _arr(g3, dom))
        # uneven splits of the deterministic tree: rank r holds items [c_r, c_{r+1})
        dets = {}
        for seed in range(3):
            cuts = np.sort(np.random.default_rng(seed).integers(0, n_total + 1, world - 1))
            b = [0] + list(cuts) + [n_total]
            t = utilities.allreduce_sum(vals[b[rank]:b[rank + 1]], comm, deterministic=True,
                                        template=lambda: 0 * mean)
            dets[seed] = _arr(t, dom)
        res["dets"] = dets
        comm.Barrier()
        dist.destroy_process_group()
        q.put((rank, res))
    except Exception as e:  # surface the failure in the parent
        import traceback
        q.put((rank, "ERROR " + repr(e) + "\n" + traceback.format_exc()))


@pytest.fixture(scope="module", params=sorted(CASES))
def world_results(request):
    world = request.param
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, CASES[world], port, q)) for r in range(world)]
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
    return world, out


def _serial(n_total):
    sys.path.insert(0, ROOT)
    from nifty_amd import utilities
    dom, vals = _values(n_total)
    return dom, vals, utilities


def test_share_range_partitions_mirrored_list(world_results):
    world, out = world_results
    n_total = 2 * CASES[world]
    rngs = [out[r]["range"] for r in range(world)]
    assert rngs[0][0] == 0 and rngs[-1][1] == n_total
    assert all(rngs[r][1] == rngs[r + 1][0] for r in range(world - 1))
    sizes = [b - a for a, b in rngs]
    assert max(sizes) - min(sizes) <= 1
    if world == 8:   # C4 / C5 shapes: whole pairs per rank
        assert all(s == n_total // 8 for s in sizes)
    if world == 3:   # a mirrored pair split across two ranks
        assert any(a % 2 == 1 for a, _ in rngs)


def test_deterministic_tree_bitwise(world_results):
    world, out = world_results
    dom, vals, utilities = _serial(2 * CASES[world])
    serial = utilities.pairwise_sum(vals)
    for r in range(world):
        for k in dom.keys():
            np.testing.assert_array_equal(out[r]["det"][k], np.asarray(serial[k]))
            np.testing.assert_allclose(out[r]["fast"][k], np.asarray(serial[k]), rtol=1e-12, atol=1e-300)
            np.testing.assert_array_equal(out[r]["fast"][k], out[0]["fast"][k])
        for seed, d in out[r]["dets"].items():
            for k in dom.keys():
                np.testing.assert_array_equal(d[k], np.asarray(serial[k]), err_msg=f"split {seed}")


def test_kl_mean_bitwise_single_process(world_results):
    """deterministic mode: the KL value / gradient mean and the sample average
    equal the one-process sample list's bit for bit on every rank"""
    world, out = world_results
    n_total = 2 * CASES[world]
    dom, vals, utilities = _serial(n_total)
    import nifty_amd as ift
    mean = vals[0]
    utilities.DETERMINISTIC_ALLREDUCE = True
    try:
        sl = ift.ResidualSampleList(mean, vals, [(i % 2) == 1 for i in range(n_total)], None)
        v1, g1 = sl._average_tuple(lambda s: (float(np.asarray(s["b"])), s))
        a1 = sl.average()
    finally:
        utilities.DETERMINISTIC_ALLREDUCE = False
    for r in range(world):
        v, g, ncall = out[r]["kl1"]
        assert v == v1
        for k in dom.keys():
            np.testing.assert_array_equal(g[k], np.asarray(g1[k]))
            np.testing.assert_array_equal(out[r]["avg1"][k], np.asarray(a1[k]))
        # fast mode: ONE collective per KL mean, equal to rounding
        vf, gf, nf = out[r]["kl0"]
        assert nf == 1
        assert vf == pytest.approx(v1, rel=1e-12, abs=1e-300)
        for k in dom.keys():
            np.testing.assert_allclose(gf[k], np.asarray(g1[k]), rtol=1e-11, atol=1e-300)


def test_ranks_without_samples(world_results):
    world, out = world_results
    dom, vals, utilities = _serial(2 * CASES[world])
    mean = vals[0]
    ref = utilities.pairwise_sum([mean + v for v in vals[:3]])
    for r in range(world):
        n, v, g = out[r]["few"]
        assert n == (1 if r < 3 else 0)
        assert v == pytest.approx(float(np.asarray(ref["b"])) / 3, rel=1e-14)
        for k in dom.keys():
            np.testing.assert_array_equal(g[k], np.asarray(ref[k]) / 3)
