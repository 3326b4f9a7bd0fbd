"""CPU: the multi-process path (one process per GPU on the box) with the gloo
backend, world_size 2 -- sample sharding (shareRange over mirrored samples),
the KL-mean all-reduce (fast: local pairwise sum + ONE all_reduce of a packed
fp64 buffer; deterministic: the reference's global pairwise tree,
bit-identical to the serial result, src/utilities.py:331-390), sample-list
averaging and the communicator wrapper.  No GPU compute."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _values(n_total):
    """per-sample MultiFields with awkward magnitudes (order-sensitive sums)"""
    import nifty_amd as ift
    dom = ift.makeDomain({"a": ift.RGSpace(7), "b": ift.DomainTuple.scalar_domain(),
                          "xi": ift.RGSpace((4, 6))})
    rng = np.random.default_rng(11)
    out = []
    for i in range(n_total):
        d = {k: rng.standard_normal(dom[k].shape) * 10.0 ** rng.integers(-8, 8, dom[k].shape)
             for k in dom.keys()}
        out.append(ift.MultiField.from_dict({k: ift.makeField(dom[k], v) for k, v in d.items()}, dom))
    return dom, out


def _worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
        sys.path.insert(0, ROOT)
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import nifty_amd as ift
        from nifty_amd import utilities
        comm = ift.TorchComm()
        assert comm.Get_rank() == rank and comm.Get_size() == world
        res = {}
        # mirrored sample list sharded as draw_samples does (kl_energies.py:140-141)
        nsamp = 5
        lo, hi = utilities.shareRange(2 * nsamp, world, rank)
        res["range"] = (lo, hi)
        n_total = 2 * nsamp
        dom, vals = _values(n_total)
        mine = vals[lo:hi]
        fast = utilities.allreduce_sum(mine, comm, deterministic=False)
        det = utilities.allreduce_sum(mine, comm, deterministic=True)
        res["fast"] = {k: np.asarray(fast[k]) for k in dom.keys()}
        res["det"] = {k: np.asarray(det[k]) for k in dom.keys()}
        # sample list averaging (mean +/- residual, mirrored signs)
        mean = vals[0]
        neg = [(i % 2) == 1 for i in range(lo, hi)]
        sl = ift.ResidualSampleList(mean, vals[lo:hi], neg, comm)
        assert sl.n_samples == n_total and sl.n_local_samples == hi - lo
        avg = sl.average()
        res["avg"] = {k: np.asarray(avg[k]) for k in dom.keys()}
        # scalar tuple averaging (value, gradient) as SampledKLEnergyClass uses it
        val, grad = sl._average_tuple(lambda s: (float(np.asarray(s["b"])), s))
        res["tuple"] = (val, {k: np.asarray(grad[k]) for k in dom.keys()})
        res["bcast"] = comm.bcast(rank * 7 + 3, root=0)
        # ONE collective per KL value + gradient mean (sample_list._average_results)
        calls = []
        orig = comm.allreduce_tensor_
        comm.allreduce_tensor_ = lambda t: (calls.append(t.numel()), orig(t))[1]
        sl._average_tuple(lambda s: (float(np.asarray(s["b"])), s))
        comm.allreduce_tensor_ = orig
        res["ncoll"] = len(calls)
        # a rank without samples (reference: the _active_comm split,
        # sample_list.py:62-70): rank 1 holds none of the 3 samples
        few = vals[:3] if rank == 0 else []
        sl0 = ift.ResidualSampleList(mean, few, [False] * len(few), comm)
        assert sl0.n_samples == 3
        zero = lambda: (0.0, 0 * mean)  # noqa: E731
        for det in (False, True):
            utilities.DETERMINISTIC_ALLREDUCE = det
            v0, g0 = sl0._average_tuple(lambda s: (float(np.asarray(s["b"])), s), zero)
            a0 = sl0.average()
            res[f"empty{int(det)}"] = (v0, {k: np.asarray(g0[k]) for k in dom.keys()},
                                       {k: np.asarray(a0[k]) for k in dom.keys()})
        utilities.DETERMINISTIC_ALLREDUCE = False
        # the deterministic tree with uneven splits: every split of 10 items
        dets = {}
        for n0 in (0, 1, 4, 7, 10):
            mine = vals[:n0] if rank == 0 else vals[n0:]
            t = utilities.allreduce_sum(mine, comm, deterministic=True, template=lambda: 0 * mean)
            dets[n0] = {k: np.asarray(t[k]) for k in dom.keys()}
        res["dets"] = dets
        comm.Barrier()
        dist.destroy_process_group()
        q.put((rank, res))
    except Exception as e:  # surface the failure in the parent
        import traceback
        q.put((rank, "ERROR " + repr(e) + "\n" + traceback.format_exc()))


@pytest.fixture(scope="module")
def results():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        r, res = q.get(timeout=240)
        out[r] = res
    for p in procs:
        p.join(timeout=60)
    for r, res in out.items():
        assert not isinstance(res, str), res
    return out


def test_share_range_covers_mirrored_samples(results):
    rngs = sorted(results[r]["range"] for r in results)
    assert rngs[0][0] == 0 and rngs[-1][1] == 10
    assert rngs[0][1] == rngs[1][0]


def test_allreduce_fast_and_deterministic(results):
    sys.path.insert(0, ROOT)
    from nifty_amd import utilities
    dom, vals = _values(10)
    serial = utilities.pairwise_sum(vals)
    for r in results:
        for k in dom.keys():
            ref = np.asarray(serial[k])
            # deterministic mode: the reference's global tree, bit for bit
            np.testing.assert_array_equal(results[r]["det"][k], ref)
            # fast mode: same value up to summation order
            np.testing.assert_allclose(results[r]["fast"][k], ref, rtol=1e-12, atol=1e-300)
            # identical on every rank
            np.testing.assert_array_equal(results[r]["fast"][k], results[0]["fast"][k])


def test_sample_list_average_over_ranks(results):
    sys.path.insert(0, ROOT)
    dom, vals = _values(10)
    mean = vals[0]
    full = [mean - v if i % 2 else mean + v for i, v in enumerate(vals)]
    for r in results:
        for k in dom.keys():
            ref = sum(np.asarray(f[k]) for f in full) / 10
            np.testing.assert_allclose(results[r]["avg"][k], ref, rtol=1e-10, atol=1e-300)
        val, grad = results[r]["tuple"]
        assert val == pytest.approx(float(np.mean([np.asarray(f["b"]) for f in full])), rel=1e-10)
        np.testing.assert_allclose(grad["xi"], results[r]["avg"]["xi"], rtol=1e-12, atol=1e-300)
    assert results[0]["bcast"] == results[1]["bcast"] == 3


def test_one_collective_per_kl_mean(results):
    """value and gradient travel in ONE packed all-reduce"""
    for r in results:
        assert results[r]["ncoll"] == 1


def test_rank_without_samples(results):
    """3 samples on 2 ranks, rank 1 holding none: both ranks get the mean of
    the 3 (fast and deterministic mode), as the reference's _active_comm +
    broadcast gives"""
    sys.path.insert(0, ROOT)
    from nifty_amd import utilities
    dom, vals = _values(10)
    mean = vals[0]
    full = [mean + v for v in vals[:3]]
    ref = utilities.pairwise_sum(full)
    for det in (0, 1):
        for r in results:
            v0, g0, a0 = results[r][f"empty{det}"]
            assert v0 == pytest.approx(float(np.asarray(ref["b"])) / 3, rel=1e-14)
            for k in dom.keys():
                np.testing.assert_allclose(g0[k], np.asarray(ref[k]) / 3, rtol=1e-13, atol=1e-300)
                np.testing.assert_allclose(a0[k], np.asarray(ref[k]) / 3, rtol=1e-13, atol=1e-300)
            if det:
                for k in dom.keys():
                    np.testing.assert_array_equal(g0[k], np.asarray(ref[k]) / 3)


def test_deterministic_tree_any_split(results):
    """the point-to-point pairwise tree equals the serial pairwise sum bit for
    bit for every split of the items over the ranks (src/utilities.py:331-390)"""
    sys.path.insert(0, ROOT)
    from nifty_amd import utilities
    dom, vals = _values(10)
    serial = utilities.pairwise_sum(vals)
    for r in results:
        for n0, d in results[r]["dets"].items():
            for k in dom.keys():
                np.testing.assert_array_equal(d[k], np.asarray(serial[k]), err_msg=f"split {n0}")


def _worker_lists(rank, world, port, q, tmp):
    """a MAP SampleList (one sample on two ranks) saved, resumed and averaged;
    the deterministic tree over fp32 and complex fields"""
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
        sys.path.insert(0, ROOT)
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import nifty_amd as ift
        from nifty_amd import utilities
        comm = ift.TorchComm()
        res = {}
        dom, vals = _values(3)
        # MAP: rank 0 holds the single sample, rank 1 none (optimize_kl's
        # SampleList of one position)
        mine = vals[:1] if rank == 0 else []
        sl = ift.SampleList(mine, comm=comm, domain=dom)
        base = os.path.join(tmp, "map")
        sl.save(base)
        back = ift.SampleList.load(base, comm=comm)   # no domain: read from sample 0's file
        res["n"] = (back.n_samples, back.n_local_samples)
        res["dom"] = back.domain == dom
        avg = back.average()
        res["avg"] = {k: np.asarray(avg[k]) for k in dom.keys()}
        op = lambda s: 2. * s["a"]  # noqa: E731  (op changes the layout)
        res["avg_op"] = np.asarray(back.average(op).val)
        m, v = back.sample_stat()
        res["stat"] = {k: np.asarray(m[k]) for k in dom.keys()}
        # the deterministic tree for fp32 and complex: bitwise the serial sum
        d2 = ift.makeDomain({"f": ift.RGSpace(9), "c": ift.RGSpace((3, 4))})
        rng = np.random.default_rng(3)
        items = []
        for i in range(7):
            f = (rng.standard_normal(9) * 10.0 ** rng.integers(-4, 4, 9)).astype(np.float32)
            c = rng.standard_normal((3, 4)) * 10.0 ** rng.integers(-6, 6, (3, 4)) \
                + 1j * rng.standard_normal((3, 4))
            items.append(ift.MultiField.from_dict({"f": ift.makeField(d2["f"], f),
                                                   "c": ift.makeField(d2["c"], c)}, d2))
        lo, hi = utilities.shareRange(7, world, rank)
        t = utilities.allreduce_sum(items[lo:hi], comm, deterministic=True)
        res["det32c"] = {k: np.asarray(t[k]) for k in d2.keys()}
        # a complex field packed after an odd count of fp64 elements (energy
        # value, complex field): odd storage offset in the shared buffer
        tup = [(float(i) + 0.25, ift.makeField(d2["c"], np.asarray(items[i]["c"].val.cpu())))
               for i in range(7)]
        res["odd"] = {}
        for det in (False, True):
            v, f = utilities.allreduce_sum(tup[lo:hi], comm, deterministic=det)
            res["odd"][det] = (v, np.asarray(f.val.cpu()))
        # fp32 / complex samples on rank 0 only: rank 1's zero template takes
        # the samples' dtypes (same collectives on both ranks)
        sl2 = ift.SampleList(items[:1] if rank == 0 else [], comm=comm, domain=d2)
        res["avg32c"] = {}
        for det in (False, True):
            utilities.DETERMINISTIC_ALLREDUCE, keep = det, utilities.DETERMINISTIC_ALLREDUCE
            try:
                a = sl2.average()
            finally:
                utilities.DETERMINISTIC_ALLREDUCE = keep
            res["avg32c"][det] = {k: np.asarray(a[k].val.cpu()) for k in d2.keys()}
        comm.Barrier()
        dist.destroy_process_group()
        q.put((rank, res))
    except Exception as e:
        import traceback
        q.put((rank, "ERROR " + repr(e) + "\n" + traceback.format_exc()))


@pytest.fixture(scope="module")
def list_results(tmp_path_factory):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    tmp = str(tmp_path_factory.mktemp("lists"))
    procs = [ctx.Process(target=_worker_lists, args=(r, world, port, q, tmp)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        r, res = q.get(timeout=240)
        out[r] = res
    for p in procs:
        p.join(timeout=60)
    for r, res in out.items():
        assert not isinstance(res, str), res
    return out


def test_map_sample_list_resume(list_results):
    """SampleList.load on a rank whose share of the files is empty takes the
    domain from sample 0's file and joins the constructor's allgather (no hang);
    average / sample_stat on that rank match the owner's"""
    _, vals = _values(3)
    assert list_results[0]["n"] == (1, 1) and list_results[1]["n"] == (1, 0)
    for r in list_results:
        assert list_results[r]["dom"]
        for k, v in list_results[r]["avg"].items():
            np.testing.assert_array_equal(v, np.asarray(vals[0][k]))
            np.testing.assert_array_equal(list_results[r]["stat"][k], np.asarray(vals[0][k]))
        np.testing.assert_array_equal(list_results[r]["avg_op"], 2. * np.asarray(vals[0]["a"]))


def test_deterministic_tree_fp32_complex(list_results):
    """fp32 stays fp32 and complex stays complex through the packed buffers:
    bitwise the serial pairwise sum on every rank"""
    sys.path.insert(0, ROOT)
    import nifty_amd as ift
    from nifty_amd import utilities
    d2 = ift.makeDomain({"f": ift.RGSpace(9), "c": ift.RGSpace((3, 4))})
    rng = np.random.default_rng(3)
    items = []
    for i in range(7):
        f = (rng.standard_normal(9) * 10.0 ** rng.integers(-4, 4, 9)).astype(np.float32)
        c = rng.standard_normal((3, 4)) * 10.0 ** rng.integers(-6, 6, (3, 4)) + 1j * rng.standard_normal((3, 4))
        items.append(ift.MultiField.from_dict({"f": ift.makeField(d2["f"], f),
                                               "c": ift.makeField(d2["c"], c)}, d2))
    serial = utilities.pairwise_sum(items)
    for r in list_results:
        for k in ("f", "c"):
            got = list_results[r]["det32c"][k]
            want = np.asarray(serial[k])
            assert got.dtype == want.dtype, (k, got.dtype)
            np.testing.assert_array_equal(got, want)


def test_allreduce_complex_odd_offset(list_results):
    """(scalar, complex field) tuples: the complex run starts at an odd offset
    of the packed fp64 buffer; both reduction modes rebuild it"""
    sys.path.insert(0, ROOT)
    import nifty_amd as ift
    from nifty_amd import utilities
    d2 = ift.makeDomain({"f": ift.RGSpace(9), "c": ift.RGSpace((3, 4))})
    rng = np.random.default_rng(3)
    cs = []
    for i in range(7):
        rng.standard_normal(9), rng.integers(-4, 4, 9)
        cs.append(rng.standard_normal((3, 4)) * 10.0 ** rng.integers(-6, 6, (3, 4)) + 1j * rng.standard_normal((3, 4)))
    tup = [(float(i) + 0.25, ift.makeField(d2["c"], cs[i])) for i in range(7)]
    sv, sf = utilities.pairwise_sum(tup)
    for r in list_results:
        for det in (False, True):
            v, f = list_results[r]["odd"][det]
            assert v == sv
            assert f.dtype == np.complex128
            if det:
                np.testing.assert_array_equal(f, np.asarray(sf.val.cpu()))
            else:
                np.testing.assert_allclose(f, np.asarray(sf.val.cpu()), rtol=1e-14, atol=0)


def test_average_empty_rank_dtypes(list_results):
    """a rank without samples reduces with the samples' fp32 / complex dtypes"""
    for r in list_results:
        ref = list_results[0]["avg32c"][False]
        for det in (False, True):
            got = list_results[r]["avg32c"][det]
            assert got["f"].dtype == np.float32 and got["c"].dtype == np.complex128
            for k in ("f", "c"):
                np.testing.assert_array_equal(got[k], ref[k])


def _worker_desync(rank, world, port, q):
    """the reference's MPI consistency guards (utilities.py:434-478,
    kl_energies.py:136-137, optimize_kl.py:342-345) firing on ranks that
    disagree -- and staying quiet on ranks that agree"""
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
        sys.path.insert(0, ROOT)
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import nifty_amd as ift
        from nifty_amd import utilities
        comm = ift.TorchComm()
        res = {}

        def raises(fn):
            try:
                fn()
            except RuntimeError as e:
                return "not in sync" in str(e)
            return False
        dom, vals = _values(2)
        f = vals[0]
        # equal objects pass
        utilities.check_MPI_synced_random_state(comm)
        utilities.check_MPI_equality(f, comm, hash_=True)
        utilities.check_MPI_equality(dom, comm)
        utilities.check_MPI_equality(np.random.SeedSequence(4).spawn(3), comm)
        # one ulp on one rank, one key
        a = np.asarray(f["a"]).copy()
        if rank == 1:
            a[3] = np.nextafter(a[3], np.inf)
        g = ift.MultiField.from_dict({"a": ift.makeField(dom["a"], a), "b": f["b"], "xi": f["xi"]}, dom)
        res["field"] = raises(lambda: utilities.check_MPI_equality(g, comm, hash_=True))
        # a permutation of the same values
        a2 = np.asarray(f["a"]).copy()
        if rank == 1:
            a2[[0, 1]] = a2[[1, 0]]
        g2 = ift.MultiField.from_dict({"a": ift.makeField(dom["a"], a2), "b": f["b"], "xi": f["xi"]}, dom)
        res["perm"] = raises(lambda: utilities.check_MPI_equality(g2, comm, hash_=True))
        d2 = ift.makeDomain({"a": ift.RGSpace(7, distances=1. + rank)})
        res["domain"] = raises(lambda: utilities.check_MPI_equality(d2, comm))
        res["sseq"] = raises(lambda: utilities.check_MPI_equality(
            np.random.SeedSequence(4 + rank).spawn(3), comm))
        # the random state: one extra draw on rank 1
        ift.random.push_sseq_from_seed(5)
        if rank == 1:
            ift.random.current_rng().standard_normal(1)
        res["state"] = raises(lambda: utilities.check_MPI_synced_random_state(comm))
        ift.random.pop_sseq()
        # optimize_kl refuses to start an iteration from means that differ
        sp = ift.RGSpace(8)
        lh = ift.GaussianEnergy(ift.full(sp, 1.)) @ ift.ScalingOperator(sp, 2.).ducktape("x")
        pos = ift.MultiField.from_dict({"x": ift.full(sp, 0.5 + 1e-3 * rank)})
        ift.random.push_sseq_from_seed(6)
        res["optkl"] = raises(lambda: ift.optimize_kl(
            lh, 1, 0, ift.NewtonCG(ift.GradientNormController(iteration_limit=1)), None, None,
            initial_position=pos, comm=comm))
        ift.random.pop_sseq()
        comm.Barrier()
        dist.destroy_process_group()
        q.put((rank, res))
    except Exception as e:
        import traceback
        q.put((rank, "ERROR " + repr(e) + "\n" + traceback.format_exc()))


def test_mpi_guards_fire_on_desync():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_desync, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        r, res = q.get(timeout=240)
        out[r] = res
    for p in procs:
        p.join(timeout=60)
    for r, res in out.items():
        assert not isinstance(res, str), res
        for k, v in res.items():
            assert v, (r, k)
